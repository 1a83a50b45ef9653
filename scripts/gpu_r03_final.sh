# Round-3 HEAD check on the shipped library: smoke, the whole -m gpu suite, the
# default bench line (secondary configs included), then the config-3 profile
# (rocprofv3 kernel trace + separate PMC passes, scripts/profile.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_final
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -2 $O/smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -2 $O/pytest_gpu.log; [ $s -eq 0 ] || exit $s
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench exit $s"; cut -c1-300 $O/bench.json; [ $s -eq 0 ] || exit $s
bash scripts/profile.sh r03_final_cfg3 > $O/profile.log 2>&1
s=$?; echo "profile exit $s"; tail -2 $O/profile.log
exit $s
