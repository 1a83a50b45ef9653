# HEAD check after the session restart: smoke, the whole -m gpu suite, the
# default bench line (secondary configs included), cfg3 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -3 $O/smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -4 $O/pytest_gpu.log; [ $s -eq 0 ] || exit $s
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench exit $s"; cut -c1-400 $O/bench.json; [ $s -eq 0 ] || exit $s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o kt -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 1 --no-secondary --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/$O/kt_bench.json 2> $GRAFT_REPO_ROOT/$O/kt_bench.err
s=$?; echo "kt exit $s"; exit $s
