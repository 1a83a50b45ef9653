# Round 5 GPU call 8: the 32-lane one-stream default (lzgpu_decode_dup_kernel,
# dup sliced lane kernel): smoke, the whole GPU suite, the default bench line
# (config 3 + secondary configs), and config 2 with 16 / 32 / 64 lanes per
# stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run8
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s: $(tail -1 $O/smoke.log)"; [ $s -eq 0 ] || exit $s
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest_gpu.log)"; [ $s -eq 0 ] || exit $s
