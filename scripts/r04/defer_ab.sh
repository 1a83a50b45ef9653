# Round 4: deferred output in the windowed cooperative kernels (decoded bytes
# to the LDS window only, stored to the dictionary 64+ at a time by all lanes)
# -- GPU parity of the cooperative paths, A/B against write-through
# (-DLZGPU_WIN_DEFER=0) on configs 4 and 1 and the xz leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_defer
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_xz.py \
  tests/test_cfg1.py tests/test_sessions.py tests/test_dropin_mirror.py tests/test_c_host.py \
  tests/test_coalesce.py tests/test_7z.py tests/test_sliced.py -x -v --timeout 300 --timeout-method thread -m gpu \
  > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -1 $O/pytest.log; [ $s -eq 0 ] || exit $s
run() {  # name lib env config steps extra
  env LZGPU_LIB=$2 $3 timeout -k 10 300 python bench.py --config $4 --steps $5 --warmup 1 \
    --no-cpu-baseline $6 > $O/$4_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$4 $1 r$round: $(python -c "import json;d=json.load(open('$O/$4_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  run defer "" "" cfg4 5 --no-gather || exit $?
  run nodefer $V/liblzmagpu_nodefer.so "" cfg4 5 --no-gather || exit $?
  run defer "" "" xz 5 || exit $?
  run nodefer $V/liblzmagpu_nodefer.so "" xz 5 || exit $?
  run defer "" "" cfg1 3 || exit $?
  run nodefer $V/liblzmagpu_nodefer.so "" cfg1 3 || exit $?
done
