#!/bin/bash
# GPU box: gpu tests, then the cooperative latency-regime kernel (default) vs
# LZGPU_COOP=0 on configs 2, 5, 4 and xz.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-coop}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 gpurun_out/${TAG}_pytest.log; [ $s -eq 0 ] || exit $s
for cfg in cfg2 cfg5 cfg4 xz; do
  for coop in 1 0; do
    LZGPU_COOP=$coop timeout -k 10 400 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${cfg}_$coop.json 2> gpurun_out/${TAG}_${cfg}_$coop.err
    s=$?; echo "$cfg coop=$coop exit $s: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${cfg}_$coop.json'));print(d['value'], d.get('verified'))")"
    [ $s -eq 0 ] || exit $s
  done
done
