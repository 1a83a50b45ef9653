# Round 4: the windowed cooperative builds with the checkpoint reader and the
# speculative literal stages (BulkReaderFor masks kWinBit) -- GPU parity of the
# cooperative paths, then A/B against the first window build's per-byte reader
# and serial literal tree (variant LZGPU_WIN_Q=0) and against no window
# (LZGPU_WIN=0) on configs 4 and 1 and the xz leg; config-4 region profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_winq
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_xz.py \
  tests/test_cfg1.py tests/test_sessions.py tests/test_dropin_mirror.py tests/test_c_host.py \
  tests/test_coalesce.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "coop or parity or cfg1 or session or xz or cfg4 or goldens or mirror or c_host or coalesce or walker" \
  > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -2 $O/pytest.log; [ $s -eq 0 ] || exit $s
run() {  # name lib env config extra
  env LZGPU_LIB=$2 $3 timeout -k 10 300 python bench.py --config $4 --steps $5 --warmup 1 \
    --no-cpu-baseline $6 > $O/$4_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$4 $1 r$round: $(python -c "import json;d=json.load(open('$O/$4_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  run q "" "" cfg4 5 --no-gather || exit $?
  run plain $V/liblzmagpu_winplain.so "" cfg4 5 --no-gather || exit $?
  run nowin "" "LZGPU_WIN=0" cfg4 5 --no-gather || exit $?
  run q "" "" xz 5 || exit $?
  run plain $V/liblzmagpu_winplain.so "" xz 5 || exit $?
  run nowin "" "LZGPU_WIN=0" xz 5 || exit $?
  run q "" "" cfg1 3 || exit $?
  run plain $V/liblzmagpu_winplain.so "" cfg1 3 || exit $?
  run nowin "" "LZGPU_WIN=0" cfg1 3 || exit $?
done
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-gather > $O/prof_cfg4.json 2> $O/prof_cfg4.err || exit $?
echo "prof: $(grep PROF $O/prof_cfg4.err | cut -c1-1200)"
# one-lane waves at one wave per SIMD (1,024 config-2 streams, 4 per CU):
# vector vs scalar-register build, and the cooperative kernel the planner picks
for round in 1 2; do
  for q in 0 4; do
    LZGPU_KERNEL=latency LZGPU_SCALAR=$q timeout -k 10 300 python bench.py --config cfg2 --streams 1024 \
      --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-crc > $O/cfg2s1k_lat_q${q}_r$round.json 2>> $O/ab.err || exit $?
    echo "cfg2x1024 latency scalar=$q r$round: $(python -c "import json;d=json.load(open('$O/cfg2s1k_lat_q${q}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
  done
  timeout -k 10 300 python bench.py --config cfg2 --streams 1024 --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc > $O/cfg2s1k_auto_r$round.json 2>> $O/ab.err || exit $?
  echo "cfg2x1024 auto(coop) r$round: $(python -c "import json;d=json.load(open('$O/cfg2s1k_auto_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
done
