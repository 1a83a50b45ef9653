#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the decoder's access shapes (run via
# gpurun; the binary is built in the container:
#   hipcc -O3 --offload-arch=gfx950 -o scripts/ubench/traffic_calib scripts/ubench/traffic_calib.hip)
# Each counter in a pass of its own; output gpurun_out/calib/<kernel>_<pass>/.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/calib"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/scripts/ubench/traffic_calib"
for k in st1 st8u st16 ld1 ld16; do
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 60 rocprofv3 --pmc $pmc -d "$OUT/${k}_$pmc" -o pmc --output-format csv -- "$B" $k \
      > "$OUT/${k}_$pmc.log" 2>&1 || exit $?
  done
  timeout -k 10 60 rocprofv3 --kernel-trace --stats -d "$OUT/${k}_kt" -o kt --output-format csv -- "$B" $k \
    > "$OUT/${k}_kt.log" 2>&1 || exit $?
  echo "calib $k done"
done
