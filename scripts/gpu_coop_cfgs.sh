#!/bin/bash
# GPU box: gpu tests, then configs 4 and xz (cooperative kernel) and 2 / 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-coopc}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 gpurun_out/${TAG}_pytest.log; [ $s -eq 0 ] || exit $s
for cfg in ${CFGS:-cfg4 xz}; do
  timeout -k 10 400 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${cfg}.json 2> gpurun_out/${TAG}_${cfg}.err
  s=$?; echo "$cfg exit $s: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${cfg}.json'));print(d['value'], d.get('verified'), d['config'].get('kernel_ms'))")"
  [ $s -eq 0 ] || exit $s
done
