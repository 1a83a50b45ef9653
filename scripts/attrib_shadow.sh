#!/bin/bash
# Write-traffic attribution for config 3, run through gpurun.
#   bash scripts/attrib_shadow.sh TAG
# Two builds of the same kernel: the default library and the attribution
# build lib/variants/liblzmagpu_shadow.so (-DLZGPU_SHADOW_OUT=512 MiB: every
# output store repeated 512 MiB further on, into room bench.py reserves with
# LZGPU_SHADOW_BYTES).  FETCH_SIZE and WRITE_SIZE in passes of their own for
# each; the WRITE_SIZE increase of the shadow build is the output's share.
set -o pipefail
TAG=${1:-attrib}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/attrib_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BARGS="--no-cpu-baseline --no-e2e --no-crc --no-secondary"
for v in default shadow; do
  if [ $v = shadow ]; then
    export LZGPU_LIB="$R/lzma-sdk-zliblike_amd/lib/variants/liblzmagpu_shadow.so"
    export LZGPU_SHADOW_BYTES=536870912
  fi
  mkdir -p "$OUT/$v"
  echo "== $v kernel trace"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/$v/kt" -o kt --output-format csv -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 $BARGS > "$OUT/$v/kt_bench.json" 2> "$OUT/$v/kt_bench.err" || exit $?
  n=0
  for pmc in FETCH_SIZE WRITE_SIZE "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
    n=$((n+1))
    echo "== $v pmc pass $n: $pmc"
    timeout -k 10 300 rocprofv3 --pmc $pmc -d "$OUT/$v/pmc$n" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 $BARGS > "$OUT/$v/pmc$n.json" 2> "$OUT/$v/pmc$n.err" || exit $?
  done
done
echo "attribution done"
