# Round 4: the cooperative kernel without a window (8 LZMA2 blocks per CU: the
# latency placement, checkpoint reader): speculative literal stages (base) vs
# the serial tree (variant qserial, LZGPU_COOP_SPEC=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_coop8
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
for round in 1 2; do
  for v in base qserial; do
    L=""; [ $v != base ] && L=$V/liblzmagpu_$v.so
    LZGPU_LIB=$L timeout -k 10 300 python bench.py --config cfg4 --blocks 2048 --steps 3 --warmup 1 \
      --no-cpu-baseline --no-gather > $O/cfg4b2048_${v}_r$round.json 2>> $O/ab.err || exit $?
    echo "cfg4x2048 $v r$round: $(python -c "import json;d=json.load(open('$O/cfg4b2048_${v}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'], d['config'].get('kernel_plan'))")"
  done
done
