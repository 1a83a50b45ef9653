set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -3 gpurun_out/smoke.log
[ $s -eq 0 ] || exit $s
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -15 gpurun_out/pytest_gpu.log
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
s=$?; echo "bench exit $s"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
exit $s
