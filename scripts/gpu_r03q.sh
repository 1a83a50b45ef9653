# Round-3 profile of the cooperative kernel on the shipped binary (config 4,
# 1,024 x 1 MiB LZMA2 blocks: rocprofv3 kernel trace + the PMC passes of
# scripts/profile.sh); then the checkpointed matched-literal variant (mlck:
# the all-LDS cooperative table's matched-literal bits decided without a refill
# check, checkpoints as in the plain tree): GPU suite on it, A/B against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
bash scripts/profile.sh r03_final_cfg4 --config cfg4 > gpurun_out/r03q_cfg4.log 2>&1
s=$?; echo "cfg4 profile exit $s"; tail -2 gpurun_out/r03q_cfg4.log; [ $s -eq 0 ] || exit $s
mkdir -p gpurun_out/r03q
LZGPU_LIB=$V/liblzmagpu_mlck.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r03q/pytest_mlck.log 2>&1
s=$?; echo "pytest mlck exit $s"; tail -1 gpurun_out/r03q/pytest_mlck.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2; do
  pts+=("cfg4::LZGPU_LIB=$V/liblzmagpu_head.so" "cfg4::LZGPU_LIB=$V/liblzmagpu_mlck.so")
  pts+=("xz::LZGPU_LIB=$V/liblzmagpu_head.so" "xz::LZGPU_LIB=$V/liblzmagpu_mlck.so")
done
bash scripts/gpu_points.sh r03q/ab "${pts[@]}"
