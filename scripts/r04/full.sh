# Round 4 HEAD check: smoke, the whole -m gpu suite, the default bench line
# (secondary configs included), then the config-3 profile (kernel trace + PMC).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_full}
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -1 $O/smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -1 $O/pytest_gpu.log; [ $s -eq 0 ] || exit $s
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench exit $s"; cut -c1-300 $O/bench.json; [ $s -eq 0 ] || exit $s
if [ "${2:-}" = "prof" ]; then
  bash scripts/profile.sh ${1:-r04_full}_cfg3 > $O/profile.log 2>&1
  s=$?; echo "profile exit $s"; tail -1 $O/profile.log
fi
exit $s
