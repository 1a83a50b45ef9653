# the cooperative kernel's match-path trees from batched LDS loads (cbatch,
# LZGPU_COOP_BATCH=1): cooperative parity tests on it, then A/B against HEAD
# on configs 4, xz and 1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
mkdir -p gpurun_out/r03v
LZGPU_LIB=$V/liblzmagpu_cbatch.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_cfg1.py \
  tests/test_gpu_parity.py tests/test_xz.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "coop or cfg1 or cfg4 or streaming or golden or xz" > gpurun_out/r03v/pytest_cbatch.log 2>&1
s=$?; echo "pytest exit $s"; tail -1 gpurun_out/r03v/pytest_cbatch.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2; do
  for v in head cbatch; do pts+=("cfg4::LZGPU_LIB=$V/liblzmagpu_$v.so" "xz::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
done
bash scripts/gpu_points.sh r03v/ab "${pts[@]}"
