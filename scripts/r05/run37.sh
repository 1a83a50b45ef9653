# Round 5 GPU call 37: the literal batch for the 32-lane one-stream kernel
# (configs 2 and 5): 4 / 8 / 16 / 32 literals per pass, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run37
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/liblzmagpu_lb4.so $V/liblzmagpu_lb16.so $V/liblzmagpu_lb32.so > $O/binary.sha256
run() {  # cfg tag lib
  local c=$1 t=$2 L=$3
  LZGPU_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/${c}_$t.json 2>> $O/ab.err || return $?
  echo "$c $t: $(python -c "import json;d=json.load(open('$O/${c}_$t.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for r in 1 2; do
  for c in cfg2 cfg5; do
    run $c lb8_r$r "" || exit $?
    run $c lb4_r$r $V/liblzmagpu_lb4.so || exit $?
    run $c lb16_r$r $V/liblzmagpu_lb16.so || exit $?
    run $c lb32_r$r $V/liblzmagpu_lb32.so || exit $?
  done
done
