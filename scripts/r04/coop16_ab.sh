# Round 4: with the cooperative kernel's literal speculation retired, the
# cooperative kernel on the latency configs (16 streams per CU, placement
# 0x1BF | coop, checkpoint reader) vs the one-lane waves the planner picks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_coop16
mkdir -p $O
run() {  # name env config
  env $2 timeout -k 10 300 python bench.py --config $3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-crc \
    > $O/$3_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$3 $1 r$round: $(python -c "import json;d=json.load(open('$O/$3_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'], d['config'].get('kernel_plan'))")"
}
for round in 1 2; do
  run base "" cfg2 || exit $?
  run coop "LZGPU_COOP=1" cfg2 || exit $?
  run base "" cfg5 || exit $?
  run coop "LZGPU_COOP=1" cfg5 || exit $?
done
