# Round 5 GPU call 19: the coalescer with concurrency gated on active callers
# (threads inside a call < half the CUs): parity tests, then 16 / 256 LzmaDecode
# and DecodeToBuf callers at the default 4 sets (256: twice) and at 1 set,
# then the coalesce bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run19
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 600 python -u -m pytest tests/test_coalesce.py tests/test_dropin_mirror.py tests/test_c_host.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest.log)"; [ $s -eq 0 ] || exit $s
F=$(python scripts/r05/stream_set.py $O/set 4096) || exit 1
B=$GRAFT_REPO_ROOT/tests/c_host/build/lzma_c_threads
for m in one buf; do
  for cfg in "16 4 a" "256 4 a" "256 4 b" "256 1 a"; do
    set -- $cfg
    LZGPU_COALESCE_INFLIGHT=$2 timeout -k 10 150 $B $1 $F 3 $m > /dev/null 2> $O/${m}_t$1_k$2_$3.err
    s=$?; echo "$m threads $1 inflight $2 ($3) exit $s: $(tail -1 $O/${m}_t$1_k$2_$3.err | cut -c1-300)"; [ $s -eq 0 ] || exit $s
  done
done
timeout -k 10 600 python -u bench.py --config coalesce > $O/coalesce.json 2> $O/coalesce.err
s=$?; echo "coalesce exit $s"; exit $s
