# throughput-kernel copy with the next matched byte from the copy's own loads
# (lz_copy<true>) and deferred probability stores (LZGPU_DEFER): GPU suite on the latter, then cfg3 A/B against the cooperative-copy
# build (coopcopy) and the HEAD build (base); region profile of cfg3 (HEAD build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r03n
mkdir -p $O
LZGPU_LIB=$V/liblzmagpu_defer.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 $O/pytest_gpu.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2 3; do
  pts+=("cfg3::LZGPU_LIB=$V/liblzmagpu_coopcopy.so" "cfg3::LZGPU_LIB=$V/liblzmagpu_mbc2.so" "cfg3::LZGPU_LIB=$V/liblzmagpu_defer.so")
done
bash scripts/gpu_points.sh r03n/ab "${pts[@]}" || exit $?
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-secondary \
  --no-cpu-baseline --no-e2e --no-crc > $O/prof_cfg3.json 2> $O/prof_cfg3.err
s=$?; echo "prof exit $s"; grep PROF $O/prof_cfg3.err | cut -c1-1200
exit $s
