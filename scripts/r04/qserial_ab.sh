# Round 4: the windowed cooperative kernels' reader once more, on the shipped
# state: per-byte reader + serial literal tree (base) vs checkpoint reader +
# serial literal tree (qserial: LZGPU_WIN_Q=1, LZGPU_COOP_SPEC=0) vs checkpoint
# reader + speculative stages (qspec: LZGPU_WIN_Q=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_qserial
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
run() {  # name lib env config steps extra
  env LZGPU_LIB=$2 $3 timeout -k 10 300 python bench.py --config $4 --steps $5 --warmup 1 \
    --no-cpu-baseline $6 > $O/$4_$1_r$round.json 2>> $O/ab.err || return $?
  echo "$4 $1 r$round: $(python -c "import json;d=json.load(open('$O/$4_$1_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  for v in base qserial qspec; do
    L=""; [ $v != base ] && L=$V/liblzmagpu_$v.so
    run $v "$L" "" cfg4 5 --no-gather || exit $?
    run $v "$L" "" xz 5 || exit $?
    run $v "$L" "" cfg1 3 || exit $?
  done
done
