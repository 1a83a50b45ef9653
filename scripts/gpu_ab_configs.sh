#!/bin/bash
# GPU box: gpu parity tests, then the default library vs a variant on
# configs 3, 2 and 5, then one profiling-build run (region cycles).
#   VARIANT=r16 PROFV=qprof bash scripts/gpu_ab_configs.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-abc}
V=${VARIANT:-r16}
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -2 gpurun_out/${TAG}_pytest.log; [ $s -eq 0 ] || exit $s
COMBOS="main:0:0 $V:0:0" bash scripts/gpu_ab.sh ${TAG}_c3 || exit 1
COMBOS="main:0:0 $V:0:0" bash scripts/gpu_ab.sh ${TAG}_c2 --config cfg2 || exit 1
COMBOS="main:0:0 $V:0:0" bash scripts/gpu_ab.sh ${TAG}_c5 --config cfg5 || exit 1
if [ -n "$PROFV" ]; then
  LZGPU_LIB=$PWD/lzma-sdk-zliblike_amd/lib/variants/liblzmagpu_$PROFV.so timeout -k 10 200 \
    python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-crc \
    > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || exit 1
  grep PROF gpurun_out/${TAG}_prof.err
fi
