# time-sliced batches: GPU parity + the cfg2 sliced leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r03e}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_sliced.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/$T/pytest_sliced.log 2>&1
s=$?; tail -30 gpurun_out/$T/pytest_sliced.log; [ $s -eq 0 ] || exit $s
for sl in 16384 65536 4096; do
  timeout -k 10 300 python -u bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-crc \
    --no-secondary --sliced $sl > gpurun_out/$T/cfg2_sliced_$sl.json 2> gpurun_out/$T/cfg2_sliced_$sl.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['kernel_avg_ms'], d['sliced'])" gpurun_out/$T/cfg2_sliced_$sl.json
done
