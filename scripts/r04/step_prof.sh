# Round 4: the decision-level loop (V2, now lz_run_step) -- per-kernel parity on
# the GPU, its config-3 kernel trace + PMC passes (LZGPU_STEP=1), the coalesced
# one-call test, and the concurrent-caller bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_stepprof
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 \
  --timeout-method thread -k "step" > $O/pytest_step.log 2>&1
s=$?; echo "pytest step exit $s"; tail -2 $O/pytest_step.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u -m pytest tests/test_coalesce.py -v --timeout 200 \
  --timeout-method thread -m gpu > $O/pytest_coalesce.log 2>&1
s=$?; echo "pytest coalesce exit $s"; tail -2 $O/pytest_coalesce.log; [ $s -eq 0 ] || exit $s
LZGPU_STEP=1 bash scripts/profile.sh r04_step_cfg3 > $O/profile.log 2>&1
s=$?; echo "profile exit $s"; tail -2 $O/profile.log; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python -u bench.py --config coalesce > $O/coalesce.json 2> $O/coalesce.err
s=$?; echo "coalesce bench exit $s"; cut -c1-600 $O/coalesce.json
exit $s
