#!/bin/bash
# Profile the bench's decode kernel on the GPU box (run through gpurun).
#   bash scripts/profile.sh TAG [bench args...]
# Writes gpurun_out/prof_TAG/: kernel-trace stats + separate PMC passes
# (counters are collected in runs of their own, never with other tracing).
set -o pipefail
TAG=${1:-r01}; shift
R="${GRAFT_REPO_ROOT:-$PWD}"
# TAG with a slash: an output directory relative to the repo (scripts/gpu.sh)
case $TAG in */*) OUT="$R/$TAG" ;; *) OUT="$R/gpurun_out/prof_$TAG" ;; esac
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BARGS="--no-cpu-baseline --no-e2e --no-crc --no-secondary $*"
sha256sum "${LZGPU_LIB:-$R/lzma-sdk-zliblike_amd/lib/liblzmagpu.so}" > "$OUT/binary.sha256"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
  python3 "$R/bench.py" --steps 5 --warmup 1 $BARGS > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err" || exit $?
n=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT"; do
  n=$((n+1))
  echo "== pmc pass $n: $pmc"
  timeout -k 10 300 rocprofv3 --pmc $pmc -d "$OUT/pmc$n" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 2 --warmup 0 $BARGS > "$OUT/pmc$n.json" 2> "$OUT/pmc$n.err" || exit $?
done
echo "profile done"
