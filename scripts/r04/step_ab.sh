# Round 4: the decision-level loop (lz_run_step) on the GPU -- per-kernel parity
# of the new instantiations, config 3 A/B against the symbol loop, then the
# round's new drop-in tests (reference LZMA2 walker, coalesced callers).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_step
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 \
  --timeout-method thread -k "step" > $O/pytest_step.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 $O/pytest_step.log; [ $s -eq 0 ] || exit $s
bash scripts/gpu_env_ab.sh r04_step/ab "LZGPU_STEP=0" "LZGPU_STEP=1" \
  "LZGPU_STEP=1 LZGPU_LANES=16 LZGPU_OCC=4 LZGPU_ILV_ANY=1" || exit $?
timeout -k 10 400 python -u -m pytest tests/test_c_host.py tests/test_coalesce.py -v --timeout 300 \
  --timeout-method thread -m gpu > $O/pytest_dropin.log 2>&1
s=$?; echo "pytest dropin exit $s"; tail -3 $O/pytest_dropin.log
exit $s
