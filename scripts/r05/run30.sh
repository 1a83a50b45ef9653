# Round 5 GPU call 30: concurrent drop-in DecodeToBuf loops against the
# oracle's traces (the suite's 120 streams, then a 400-stream campaign).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run30
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 600 python -u -m pytest tests/test_coalesce.py -v --timeout 500 --timeout-method thread -m gpu \
  -k decode_to_buf_loops_fuzz > $O/pytest_dropin_fuzz.log 2>&1
s=$?; echo "dropin fuzz exit $s: $(tail -1 $O/pytest_dropin_fuzz.log)"; [ $s -eq 0 ] || exit $s
LZGPU_DROPIN_FUZZ=400 LZGPU_DROPIN_SEED=2026 timeout -k 10 900 python -u -m pytest tests/test_coalesce.py -v \
  --timeout 850 --timeout-method thread -m gpu -k decode_to_buf_loops_fuzz > $O/dropin_fuzz_400_seed2026.log 2>&1
s=$?; echo "dropin fuzz 400 exit $s: $(tail -1 $O/dropin_fuzz_400_seed2026.log)"; exit $s
