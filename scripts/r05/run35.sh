# Round 5 GPU call: run5 (SIMD issue micro-benchmark with occupancy records,
# region profiles with tail / init counters) then run3 (the drop-in: mirror,
# ring and host-edit tests, the reference LZMA2 walker in ring mode, coalescing
# tests, the coalesce bench with its phase split, kernel traces of 1 and 16
# callers), plus the per-kernel parity matrix on the pruned build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/r05/run5.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -v --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/r05_run5/pytest_kernels.log 2>&1
s=$?; echo "pytest kernels exit $s: $(tail -1 gpurun_out/r05_run5/pytest_kernels.log)"; [ $s -eq 0 ] || exit $s
bash scripts/r05/run3.sh
