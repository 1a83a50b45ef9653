# Round 4: the packed lookahead kept for the lane kernels, the cooperative
# kernels' state held in vector registers (lz_vzero) and their windowed builds
# back on the per-byte reader -- whole GPU suite, then A/B against the
# committed r04_win state (variant winplainbytes: byte-array lookahead) on the
# cooperative configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_tmp3
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
  run winplainbytes $V/liblzmagpu_winplainbytes.so "" cfg4 5 --no-gather || exit $?
  run base "" "" xz 5 || exit $?
  run winplainbytes $V/liblzmagpu_winplainbytes.so "" xz 5 || exit $?
  run base "" "" cfg1 3 || exit $?
  run winplainbytes $V/liblzmagpu_winplainbytes.so "" cfg1 3 || exit $?
done
