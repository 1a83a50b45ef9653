# sliced leg on cfg5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r03g}
mkdir -p gpurun_out/$T
for spec in cfg5:65536 cfg5:16384; do
  c=${spec%%:*}; sl=${spec#*:}
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-crc \
    --no-secondary --sliced $sl > gpurun_out/$T/${c}_sliced_$sl.json 2> gpurun_out/$T/${c}_sliced_$sl.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['kernel_avg_ms'], d['sliced'])" gpurun_out/$T/${c}_sliced_$sl.json
done
