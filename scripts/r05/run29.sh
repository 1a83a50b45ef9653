# Round 5 GPU call 29: config-3 region profile of the fast-tail build
# (LZGPU_PROF=1 variant), and the literal batch re-checked on it (6 / 8 / 10).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run29
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/liblzmagpu_prof.so $V/liblzmagpu_lb6.so $V/liblzmagpu_lb10.so > $O/binary.sha256
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config cfg3 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-e2e --no-crc --no-secondary > $O/prof_cfg3.json 2> $O/prof_cfg3.err
s=$?; echo "prof cfg3 exit $s: $(grep PROF $O/prof_cfg3.err | cut -c1-1600)"; [ $s -eq 0 ] || exit $s
run() {  # tag lib
  local t=$1 L=$2
  LZGPU_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/cfg3_$t.json 2>> $O/ab.err || return $?
  echo "cfg3 $t: $(python -c "import json;d=json.load(open('$O/cfg3_$t.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for r in 1 2; do
  run lb8_r$r "" || exit $?
  run lb6_r$r $V/liblzmagpu_lb6.so || exit $?
  run lb10_r$r $V/liblzmagpu_lb10.so || exit $?
done
