# Round 5 GPU call 11: the coalescer with several batches in flight and one
# bulk output download per batch -- its parity tests, the coalesce bench, and
# rocprofv3 kernel traces of 1 and 16 LzmaDecode callers (run3.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run11
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_coalesce.py tests/test_dropin_mirror.py tests/test_c_host.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest.log)"; [ $s -eq 0 ] || exit $s
RUN3_OUT=$O bash scripts/r05/run3.sh
