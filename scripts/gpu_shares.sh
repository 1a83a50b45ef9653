# Strong-scaling emulation on ONE GPU: the per-GPU share of
# config 3 (65,536 / N streams) and config 2 (4,096 / N) for N = 1, 2, 4, 8, through
# the planner's default and the shapes given as extra env settings.
# usage: bash scripts/gpu_shares.sh OUTDIR ["ENV1=.. ENV2=.."]...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-shares}
shift
mkdir -p "$OUT"
VARIANTS=("" "$@")
for cfg in cfg3 cfg2; do
  if [ $cfg = cfg3 ]; then full=65536; else full=4096; fi
  for N in 1 2 4 8; do
    share=$((full / N))
    for v in "${VARIANTS[@]}"; do
      tag=$(echo "${cfg}_${share}_${v}" | tr ' =' '_-')
      env $v timeout -k 10 300 python -u bench.py --config $cfg --streams $share --steps 5 --warmup 1 \
        --no-secondary --no-e2e --no-crc --no-cpu-baseline > "$OUT/$tag.json" 2> "$OUT/$tag.err"
      s=$?
      python3 -c "
import json,sys
d=json.load(open('$OUT/$tag.json'))
r=d['roofline']; p=d['config']['kernel_plan']
print('$cfg', $share, '[$v]', d['value'], 'MB/s', r['kernel_avg_ms'], 'ms', p, d['verified'])" || echo "$tag exit $s"
      [ $s -eq 0 ] || [ $s -eq 3 ] || exit $s
    done
  done
done
