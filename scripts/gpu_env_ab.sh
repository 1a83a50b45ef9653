#!/bin/bash
# A/B of planner environment settings on the bench (run via gpurun):
#   bash scripts/gpu_env_ab.sh TAG "ENV=1 ENV2=x" "ENV=0" ... [-- bench args]
# Each setting runs twice, interleaved; prints value / kernel ms per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
[ "$1" == "--" ] && shift
for round in 1 2; do
  i=0
  for e in "${sets[@]}"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-crc "$@" \
      > gpurun_out/${TAG}_s${i}_r$round.json 2>> gpurun_out/${TAG}.err || exit $?
    echo "[$e] r$round: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_s${i}_r$round.json'));print(d['value'], d['roofline']['kernel_avg_ms'], d['verified'])")"
  done
done
