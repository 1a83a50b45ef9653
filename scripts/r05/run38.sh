# Round 5 GPU call 38: drop-in tests after lowering the call scratch's pinned
# staging floor (1 MiB -> 256 KiB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run38
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_coalesce.py tests/test_dropin_mirror.py tests/test_c_host.py \
  tests/test_gpu_parity.py tests/test_sessions.py -x -q --timeout 600 --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest.log)"; exit $s
