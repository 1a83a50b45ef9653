# Round 4: config 2's latency shape re-checked on the shipped build: one-lane
# waves x 16 per CU (default) vs 2-lane waves x 8 per CU (the two streams of a
# wave share its low-half VALU pass) and 2 x 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_latshape
mkdir -p $O
run() {  # name env config
  env $2 timeout -k 10 300 python bench.py --config $3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-crc \
    > $O/$3_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$3 $1 r$round: $(python -c "import json;d=json.load(open('$O/$3_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'], d['config'].get('kernel_plan'))")"
}
for round in 1 2; do
  run base "" cfg2 || exit $?
  run l2g8 "LZGPU_KERNEL=latency LZGPU_LANES=2 LZGPU_GROUPS=8" cfg2 || exit $?
  run l2g16 "LZGPU_KERNEL=latency LZGPU_LANES=2 LZGPU_GROUPS=16" cfg2 || exit $?
done
