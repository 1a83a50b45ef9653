# Round 4: the cooperative kernel's serial decoder on the scalar unit, now that
# the windowed builds run the serial literal tree (no speculative stages):
# base (state held in vector registers, lz_vzero) vs coopscalar
# (-DLZGPU_COOP_VREG=0) on configs 4 and 1 and the xz leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_coopscalar
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
run() {  # name lib env config steps extra
  env LZGPU_LIB=$2 $3 timeout -k 10 300 python bench.py --config $4 --steps $5 --warmup 1 \
    --no-cpu-baseline $6 > $O/$4_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$4 $1 r$round: $(python -c "import json;d=json.load(open('$O/$4_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  run base "" "" cfg4 5 --no-gather || exit $?
  run coopscalar $V/liblzmagpu_coopscalar.so "" cfg4 5 --no-gather || exit $?
  run base "" "" xz 5 || exit $?
  run coopscalar $V/liblzmagpu_coopscalar.so "" xz 5 || exit $?
  run base "" "" cfg1 3 || exit $?
  run coopscalar $V/liblzmagpu_coopscalar.so "" cfg1 3 || exit $?
done
