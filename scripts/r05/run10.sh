# Round 5 GPU call 10: configs 2 / 5 on the 32-lane one-stream kernel against
# the wave-cooperative kernel in the same latency placement (cooperative
# copies and direct bits: LZGPU_COOP=1 LZGPU_COOP_LAT=1), two rounds; the
# config-2 region profile of the 32-lane kernel (LZGPU_PROF=1 variant); then
# the drop-in measurements of run3.sh.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run10
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/liblzmagpu_prof.so > $O/binary.sha256
run() {  # cfg tag env...
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/${c}_$t.json 2>> $O/ab.err || return $?
  echo "$c $t: $(python -c "import json;d=json.load(open('$O/${c}_$t.json'));k=d['config']['kernel_plan'];print(d['value'], d['ms_per_step'], d['verified'], k.get('placement'), k.get('workgroups_per_cu'))")"
}
for r in 1 2; do
  run cfg2 dup_r$r X=1 || exit $?
  run cfg2 cooplat_r$r LZGPU_COOP=1 LZGPU_COOP_LAT=1 || exit $?
  run cfg5 dup_r$r X=1 || exit $?
  run cfg5 cooplat_r$r LZGPU_COOP=1 LZGPU_COOP_LAT=1 || exit $?
done
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config cfg2 --steps 1 --warmup 1 \
  --no-cpu-baseline --no-e2e --no-crc --no-secondary > $O/prof_cfg2.json 2> $O/prof_cfg2.err
s=$?; echo "prof cfg2 exit $s: $(grep PROF $O/prof_cfg2.err | cut -c1-1600)"; [ $s -eq 0 ] || exit $s
bash scripts/r05/run3.sh
