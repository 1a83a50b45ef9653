# Round-3 A/B, second pass.  base2 = HEAD source (uniform stores in the
# cooperative literal stage; the throughput copy back to its round-2 form after
# the next-matched-byte-from-registers variant measured -3.5 % on config 3);
# uni2 = + wave-uniform branches in the cooperative kernel and in one-lane
# latency waves (LZGPU_COOP_UNI=1 LZGPU_ONE_UNI=1); defer2 = + deferred
# probability stores in the throughput match path (LZGPU_DEFER=1).
# Parity first: the whole GPU suite on base2 and on uni2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r03p
mkdir -p $O
for v in base2 uni2; do
  LZGPU_LIB=$V/liblzmagpu_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread > $O/pytest_$v.log 2>&1
  s=$?; echo "pytest $v exit $s"; tail -1 $O/pytest_$v.log; [ $s -eq 0 ] || exit $s
done
pts=()
for rep in 1 2; do
  pts+=("cfg3::LZGPU_LIB=$V/liblzmagpu_coopcopy.so" "cfg3::LZGPU_LIB=$V/liblzmagpu_base2.so" "cfg3::LZGPU_LIB=$V/liblzmagpu_defer2.so")
  pts+=("cfg4::LZGPU_LIB=$V/liblzmagpu_base2.so" "cfg4::LZGPU_LIB=$V/liblzmagpu_uni2.so")
  pts+=("cfg2::LZGPU_LIB=$V/liblzmagpu_base2.so" "cfg2::LZGPU_LIB=$V/liblzmagpu_uni2.so")
done
pts+=("cfg5::LZGPU_LIB=$V/liblzmagpu_base2.so" "cfg5::LZGPU_LIB=$V/liblzmagpu_uni2.so")
pts+=("xz::LZGPU_LIB=$V/liblzmagpu_base2.so" "xz::LZGPU_LIB=$V/liblzmagpu_uni2.so")
bash scripts/gpu_points.sh r03p/ab "${pts[@]}"
