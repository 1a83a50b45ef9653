# A/B round: (1) throughput copy with the next matched byte from its own loads
# (mbc2 = HEAD source) and deferred probability stores (defer, LZGPU_DEFER=1)
# on config 3 against the cooperative-copy build (coopcopy); (2) the
# cooperative literal stage with uniform stores (ust, LZGPU_SPEC_UST=1) on
# config 4 against mbc2, and wave-uniform branches in the cooperative kernel
# and in one-lane latency waves (uni: LZGPU_COOP_UNI=1 LZGPU_ONE_UNI=1) on
# configs 4, xz, 2 and 5.  Parity first: the whole GPU suite on defer, the
# cooperative tests on ust.  Last: region profile of config 3 (older build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r03o
mkdir -p $O
LZGPU_LIB=$V/liblzmagpu_defer.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/pytest_defer.log 2>&1
s=$?; echo "pytest defer exit $s"; tail -2 $O/pytest_defer.log; [ $s -eq 0 ] || exit $s
LZGPU_LIB=$V/liblzmagpu_ust.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_cfg1.py \
  tests/test_sessions.py -m gpu -x -v --timeout 300 --timeout-method thread -k "coop or cfg1 or session or cfg4" \
  > $O/pytest_ust.log 2>&1
s=$?; echo "pytest ust exit $s"; tail -2 $O/pytest_ust.log; [ $s -eq 0 ] || exit $s
LZGPU_LIB=$V/liblzmagpu_uni.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/pytest_uni.log 2>&1
s=$?; echo "pytest uni exit $s"; tail -2 $O/pytest_uni.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2 3; do
  pts+=("cfg3::LZGPU_LIB=$V/liblzmagpu_coopcopy.so" "cfg3::LZGPU_LIB=$V/liblzmagpu_mbc2.so" "cfg3::LZGPU_LIB=$V/liblzmagpu_defer.so")
done
for rep in 1 2; do
  pts+=("cfg4::LZGPU_LIB=$V/liblzmagpu_mbc2.so" "cfg4::LZGPU_LIB=$V/liblzmagpu_ust.so" "cfg4::LZGPU_LIB=$V/liblzmagpu_uni.so")
done
pts+=("xz::LZGPU_LIB=$V/liblzmagpu_mbc2.so" "xz::LZGPU_LIB=$V/liblzmagpu_uni.so")
for rep in 1 2; do
  pts+=("cfg2::LZGPU_LIB=$V/liblzmagpu_mbc2.so" "cfg2::LZGPU_LIB=$V/liblzmagpu_uni.so")
done
pts+=("cfg5::LZGPU_LIB=$V/liblzmagpu_mbc2.so" "cfg5::LZGPU_LIB=$V/liblzmagpu_uni.so")
bash scripts/gpu_points.sh r03o/ab "${pts[@]}" || exit $?
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-secondary \
  --no-cpu-baseline --no-e2e --no-crc > $O/prof_cfg3.json 2> $O/prof_cfg3.err
s=$?; echo "prof exit $s"; grep PROF $O/prof_cfg3.err | cut -c1-1200
exit $s
