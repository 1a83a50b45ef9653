# Round 5 GPU call 28: the tail-truncation parity test through every kernel,
# then the coalesce bench on the final binary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run28
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread -m gpu \
  -k tail_truncations > $O/pytest_tail.log 2>&1
s=$?; echo "tail test exit $s: $(tail -1 $O/pytest_tail.log)"; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python -u bench.py --config coalesce > $O/coalesce.json 2> $O/coalesce.err
s=$?; echo "coalesce exit $s"; exit $s
