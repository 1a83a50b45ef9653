# Bench points on ONE GPU: each argument is CFG:STREAMS:"ENV=.. ENV=.." (env may be empty),
# e.g.  bash scripts/gpu_points.sh OUTDIR cfg3:8192: "cfg3:8192:LZGPU_LANES=8 LZGPU_GROUPS=4"
# One short bench run per point (--no-secondary --no-e2e --no-crc --no-cpu-baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-points}
shift
mkdir -p "$OUT"
for spec in "$@"; do
  cfg=${spec%%:*}; rest=${spec#*:}; streams=${rest%%:*}; v=${rest#*:}
  tag=$(echo "${cfg}_${streams}_${v}" | sed 's#[^ =]*/##g' | tr ' =' '_-')
  sarg=""; [ -n "$streams" ] && sarg="--streams $streams"
  env $v timeout -k 10 300 python -u bench.py --config $cfg $sarg --steps 5 --warmup 1 \
    --no-secondary --no-e2e --no-crc --no-cpu-baseline > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  s=$?
  python3 -c "
import json
d=json.load(open('$OUT/$tag.json'))
r=d.get('roofline') or {}; p=d.get('config', {}).get('kernel_plan')
print('$cfg', '$streams', '[$v]', d['value'], 'MB/s', r.get('kernel_avg_ms', d.get('ms_per_step')), 'ms', p, d['verified'])" | tee -a "$OUT/summary.log" || echo "$tag exit $s"
  [ $s -eq 0 ] || [ $s -eq 3 ] || exit $s
done
