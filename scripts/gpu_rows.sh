#!/bin/bash
# GPU box: the 8(f)-row benches (xz block batch) and configs 4/5 after a change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-rows}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 gpurun_out/${TAG}_pytest.log; [ $s -eq 0 ] || exit $s
for cfg in xz cfg4 cfg2 cfg5; do
  timeout -k 10 400 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$cfg.json 2> gpurun_out/${TAG}_$cfg.err
  s=$?; echo "$cfg exit $s"; cut -c1-600 gpurun_out/${TAG}_$cfg.json; [ $s -eq 0 ] || exit $s
done
