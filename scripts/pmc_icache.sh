#!/bin/bash
# GPU box: instruction-cache and issue counters of the decode kernel (one
# rocprofv3 --pmc pass per counter group).  bash scripts/pmc_icache.sh TAG
set -o pipefail
TAG=${1:-ic}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
n=0
for pmc in "SQC_ICACHE_MISSES" "SQC_ICACHE_REQ" "SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU"; do
  n=$((n+1))
  echo "pass $n: $pmc"
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d "$OUT/pmc$n" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --no-crc > "$OUT/pmc$n.json" 2> "$OUT/pmc$n.err" || exit $?
done
echo done
