# Round 5 GPU call 15: the group-commit coalescer with per-caller wake-ups, a
# budget of one in-flight call per CU and the resident-wave register budget
# (lone calls on the W = 2 cooperative build): parity tests, then 1 / 16 / 256
# LzmaDecode callers and 16 / 256 DecodeToBuf callers with 1 and 4 batches in
# flight, then the coalesce bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run15
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 600 python -u -m pytest tests/test_coalesce.py tests/test_dropin_mirror.py tests/test_c_host.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest.log)"; [ $s -eq 0 ] || exit $s
F=$(python scripts/r05/stream_set.py $O/set 4096) || exit 1
B=$GRAFT_REPO_ROOT/tests/c_host/build/lzma_c_threads
for m in one buf; do
  for t in 1 16 256; do
    [ $m = buf ] && [ $t = 1 ] && continue
    for k in 1 4; do
      [ $t = 1 ] && [ $k = 1 ] && continue
      r=3; [ $t = 1 ] && r=1
      LZGPU_COALESCE_INFLIGHT=$k timeout -k 10 150 $B $t $F $r $m > /dev/null 2> $O/${m}_t${t}_k$k.err
      s=$?; echo "$m threads $t inflight $k exit $s: $(tail -1 $O/${m}_t${t}_k$k.err | cut -c1-330)"; [ $s -eq 0 ] || exit $s
    done
  done
done
timeout -k 10 600 python -u bench.py --config coalesce > $O/coalesce.json 2> $O/coalesce.err
s=$?; echo "coalesce exit $s"; exit $s
