# Round 5 GPU call 3: the drop-in (ADVICE r04 items + VERDICT r04 item 4):
# the coalesce bench (phase split of a lone call) and a
# rocprofv3 kernel trace of one- and 16-caller LzmaDecode runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${RUN3_OUT:-gpurun_out/r05_run3}
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 600 python -u bench.py --config coalesce > $O/coalesce.json 2> $O/coalesce.err
s=$?; echo "coalesce exit $s: $(grep -c phase_us $O/coalesce.err) rows"; [ $s -eq 0 ] || exit $s
F=$(python scripts/r05/stream_set.py $O/set 1024) || exit 1
B=$GRAFT_REPO_ROOT/tests/c_host/build/lzma_c_threads
cd /tmp && export TMPDIR=/tmp
for t in 1 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$t -o kt --output-format csv -- \
    $B $t $F 1 one > $GRAFT_REPO_ROOT/$O/kt_$t.out 2> $GRAFT_REPO_ROOT/$O/kt_$t.err
  s=$?; echo "kt $t exit $s: $(tail -1 $GRAFT_REPO_ROOT/$O/kt_$t.err | cut -c1-600)"; [ $s -eq 0 ] || exit $s
done
