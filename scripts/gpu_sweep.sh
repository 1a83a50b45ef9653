#!/bin/bash
# Parity tests + bench variants on the GPU box (via gpurun).  Stops at the first
# crash/timeout (exit codes other than 0/1 from pytest).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-sweep}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -6 gpurun_out/${TAG}_pytest.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
s=$?; echo "bench exit $s"; cat gpurun_out/${TAG}_bench.json
[ $s -eq 0 ] || exit $s
for lv in ${SWEEP:-4:4 2:4 2:8 2:6 1:8 4:6 8:4}; do
  v=${lv%%:*}; o=${lv##*:}
  LZGPU_LANES=$v LZGPU_OCC=$o timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_l${v}o${o}.json 2>> gpurun_out/${TAG}_bench.err
  s=$?; echo "lanes=$v occ=$o exit $s: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_l${v}o${o}.json'));print(d['value'], d['ms_per_step'], d['config']['kernel_plan'], d['verified'])")"
  [ $s -eq 0 ] || exit $s
done
for cfg in ${SWEEP_CFGS:-cfg2}; do
  timeout -k 10 600 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$cfg.json 2>> gpurun_out/${TAG}_bench.err
  s=$?; echo "$cfg exit $s: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_$cfg.json'));print(d['value'], d['ms_per_step'], d['config']['kernel_plan'], d['verified'])")"
  [ $s -eq 0 ] || exit $s
done
