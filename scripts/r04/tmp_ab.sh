# Round 4: the lookahead buffer packed into registers (LzTmp) -- the decoder
# state leaves scratch memory in every kernel and the cooperative kernel's
# serial path compiles to scalar code -- plus the windowed cooperative builds
# back on the checkpoint reader.  Whole GPU suite, then A/B on the cooperative
# configs (4, 1, xz): base / tmpbytes (byte-array lookahead, -DLZGPU_TMP_BYTES=1)
# / winplainbytes (also the first window build's reader, the committed r04_win
# state) / nowin (LZGPU_WIN=0 on base).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_tmp
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -1 $O/pytest_gpu.log; [ $s -eq 0 ] || exit $s
run() {  # name lib env config steps extra
  env LZGPU_LIB=$2 $3 timeout -k 10 300 python bench.py --config $4 --steps $5 --warmup 1 \
    --no-cpu-baseline $6 > $O/$4_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$4 $1 r$round: $(python -c "import json;d=json.load(open('$O/$4_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  run base "" "" cfg4 5 --no-gather || exit $?
  run tmpbytes $V/liblzmagpu_tmpbytes.so "" cfg4 5 --no-gather || exit $?
  run winplainbytes $V/liblzmagpu_winplainbytes.so "" cfg4 5 --no-gather || exit $?
  run nowin "" "LZGPU_WIN=0" cfg4 5 --no-gather || exit $?
  run base "" "" xz 5 || exit $?
  run tmpbytes $V/liblzmagpu_tmpbytes.so "" xz 5 || exit $?
  run winplainbytes $V/liblzmagpu_winplainbytes.so "" xz 5 || exit $?
  run base "" "" cfg1 3 || exit $?
  run tmpbytes $V/liblzmagpu_tmpbytes.so "" cfg1 3 || exit $?
  run winplainbytes $V/liblzmagpu_winplainbytes.so "" cfg1 3 || exit $?
done
