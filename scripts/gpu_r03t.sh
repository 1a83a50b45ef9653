# literal batch 64 for the latency placement only (lblat = HEAD source): GPU
# suite on it, then A/B against the previous HEAD binary on configs 2, 5, the
# 8,192-stream config-3 share (2-lane latency waves) and config 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
mkdir -p gpurun_out/r03t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03t/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -1 gpurun_out/r03t/pytest_gpu.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2; do
  for v in head lblat; do pts+=("cfg2::LZGPU_LIB=$V/liblzmagpu_$v.so" "cfg5::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
done
for v in head lblat; do pts+=("cfg3:8192:LZGPU_LIB=$V/liblzmagpu_$v.so" "cfg3::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
bash scripts/gpu_points.sh r03t/ab "${pts[@]}"
