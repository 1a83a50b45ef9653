# random-byte poison vs constant fill on cfg4 / cfg3 / cfg2 (first-step effect)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03i5
for c in cfg4 cfg3 cfg2; do
  for p in rand const; do
    LZGPU_BENCH_POISON=$p timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 1 --no-cpu-baseline --no-gather \
      --no-e2e --no-crc --no-secondary > gpurun_out/r03i5/${c}_$p.json 2> gpurun_out/r03i5/${c}_$p.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['kernel_avg_ms'], r.get('kernel_ms_steps'), d['verified'])" gpurun_out/r03i5/${c}_$p.json
  done
done
