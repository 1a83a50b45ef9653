#!/bin/bash
# A/B the code-shape variant builds on one bench config (run via gpurun):
#   bash scripts/gpu_variants_cfg.sh TAG CONFIG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-var}; CFG=${2:-cfg2}
for round in 1 2; do
for so in lzma-sdk-zliblike_amd/lib/variants/*.so; do
  v=$(basename $so .so)
  LZGPU_LIB=$PWD/$so timeout -k 10 300 python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-e2e --no-crc > gpurun_out/${TAG}_${v}_$round.json 2>> gpurun_out/${TAG}.err
  s=$?; echo "$v r$round exit $s: $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
  [ $s -eq 0 ] || exit $s
done
done
