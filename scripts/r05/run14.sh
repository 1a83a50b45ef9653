# Round 5 GPU call 14: 256 concurrent LzmaDecode callers with 1, 2 and 4
# batches in flight (LZGPU_COALESCE_INFLIGHT), and a rocprofv3 kernel trace
# of the 4-in-flight run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run14
mkdir -p $O
F=$(python scripts/r05/stream_set.py $O/set 4096) || exit 1
B=$GRAFT_REPO_ROOT/tests/c_host/build/lzma_c_threads
for t in 16 256; do
  for k in 1 2 4 8; do
    LZGPU_COALESCE_INFLIGHT=$k timeout -k 10 120 $B $t $F 3 one > /dev/null 2> $O/t${t}_k$k.err
    s=$?; echo "threads $t inflight $k exit $s: $(tail -1 $O/t${t}_k$k.err | cut -c1-400)"; [ $s -eq 0 ] || exit $s
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_256 -o kt --output-format csv -- \
  $B 256 $F 1 one > $GRAFT_REPO_ROOT/$O/kt_256.out 2> $GRAFT_REPO_ROOT/$O/kt_256.err
s=$?; echo "kt 256 exit $s"; exit $s
