# Round 4: config 3's wave shape re-checked now that the decoder state is out
# of scratch (fewer spills at 128 VGPRs): 32 lanes x 2 waves per SIMD (default)
# vs 16 lanes x 4 waves per SIMD (interleaved rows half used).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_occ
mkdir -p $O
run() {  # name env
  env $2 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-crc \
    > $O/cfg3_$1_r$round.json 2>> $O/ab.err || return $?
  echo "cfg3 $1 r$round: $(python -c "import json;d=json.load(open('$O/cfg3_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  run base "" || exit $?
  run w16x4 "LZGPU_LANES=16 LZGPU_OCC=4 LZGPU_ILV_ANY=1" || exit $?
  run w16x4s "LZGPU_LANES=16 LZGPU_OCC=4" || exit $?
done
