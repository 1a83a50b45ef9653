# cooperative literal stage: each speculative path counts its normalisations
# (the window shifted once by the winner's count) instead of carrying its own
# shifted window and byte count (shn): cooperative parity tests, A/B vs HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
mkdir -p gpurun_out/r03x
LZGPU_LIB=$V/liblzmagpu_shn.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_cfg1.py \
  tests/test_gpu_parity.py tests/test_xz.py tests/test_sessions.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "coop or cfg1 or cfg4 or streaming or golden or xz or session" > gpurun_out/r03x/pytest_shn.log 2>&1
s=$?; echo "pytest exit $s"; tail -1 gpurun_out/r03x/pytest_shn.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2; do
  for v in head shn; do pts+=("cfg4::LZGPU_LIB=$V/liblzmagpu_$v.so" "xz::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
done
bash scripts/gpu_points.sh r03x/ab "${pts[@]}"
