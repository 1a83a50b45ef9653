# Round 4, second half of tmp_ab.sh: the lane kernels (configs 3, 2, 5) with
# and without the packed lookahead, one-lane waves at one wave per SIMD (vector
# vs scalar-register build), and the config-4 region profile of the new build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_tmp2
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
run() {  # name lib env config steps extra
  env LZGPU_LIB=$2 $3 timeout -k 10 300 python bench.py --config $4 --steps $5 --warmup 1 \
    --no-cpu-baseline $6 > $O/$4_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$4 $1 r$round: $(python -c "import json;d=json.load(open('$O/$4_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  run base "" "" cfg3 20 "--no-e2e --no-crc" || exit $?
  run tmpbytes $V/liblzmagpu_tmpbytes.so "" cfg3 20 "--no-e2e --no-crc" || exit $?
  run base "" "" cfg2 5 "--no-e2e --no-crc" || exit $?
  run tmpbytes $V/liblzmagpu_tmpbytes.so "" cfg2 5 "--no-e2e --no-crc" || exit $?
  run base "" "" cfg5 5 || exit $?
  run tmpbytes $V/liblzmagpu_tmpbytes.so "" cfg5 5 || exit $?
  run lowocc_vec "" "LZGPU_KERNEL=latency LZGPU_SCALAR=0" cfg2 5 "--streams 1024 --no-e2e --no-crc" || exit $?
  run lowocc_scalar "" "LZGPU_KERNEL=latency LZGPU_SCALAR=4" cfg2 5 "--streams 1024 --no-e2e --no-crc" || exit $?
  run lowocc_coop "" "" cfg2 5 "--streams 1024 --no-e2e --no-crc" || exit $?
done
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-gather > $O/prof_cfg4.json 2> $O/prof_cfg4.err || exit $?
echo "prof: $(grep PROF $O/prof_cfg4.err | cut -c1-1200)"
