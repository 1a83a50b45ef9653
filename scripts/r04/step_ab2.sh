# Round 4: decision-level loop V1 (default library) and V2 (lib/variants/
# liblzmagpu_step2.so): per-kernel parity of both, config 3 A/B against the
# symbol loop, then the round's new drop-in tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_step
mkdir -p $O
V2=$PWD/lzma-sdk-zliblike_amd/lib/variants/liblzmagpu_step2.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 \
  --timeout-method thread -k "step" > $O/pytest_step.log 2>&1
s=$?; echo "pytest v1 exit $s"; tail -2 $O/pytest_step.log; [ $s -eq 0 ] || exit $s
LZGPU_LIB=$V2 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 \
  --timeout-method thread -k "step" > $O/pytest_step2.log 2>&1
s=$?; echo "pytest v2 exit $s"; tail -2 $O/pytest_step2.log; [ $s -eq 0 ] || exit $s
bash scripts/gpu_env_ab.sh r04_step/ab "LZGPU_STEP=0" "LZGPU_STEP=1" "LZGPU_STEP=1 LZGPU_LIB=$V2" \
  "LZGPU_STEP=1 LZGPU_LIB=$V2 LZGPU_LANES=16 LZGPU_OCC=4 LZGPU_ILV_ANY=1" || exit $?
timeout -k 10 400 python -u -m pytest tests/test_c_host.py tests/test_coalesce.py -v --timeout 300 \
  --timeout-method thread -m gpu > $O/pytest_dropin.log 2>&1
s=$?; echo "pytest dropin exit $s"; tail -3 $O/pytest_dropin.log
exit $s
