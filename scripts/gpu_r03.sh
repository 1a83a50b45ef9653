# Round-3 GPU check: smoke, the -m gpu suite, the config-1 leg, the default bench line.
# usage (from the repo root on the GPU box):  bash scripts/gpu_r03.sh OUTDIR [pytest -k expr]
# Stops at the first step that faults, aborts or times out (exit 124/134/137/139);
# a plain test failure (pytest exit 1) still runs the bench steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03}
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
s=$?; echo "smoke exit $s"; tail -2 "$OUT/smoke.log"
[ $s -eq 0 ] || exit $s
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/pytest_gpu.log" 2>&1
s=$?; echo "pytest exit $s"; tail -4 "$OUT/pytest_gpu.log"
[ $s -eq 0 ] || [ $s -eq 1 ] || [ $s -eq 5 ] || exit $s
timeout -k 10 300 python -u bench.py --config cfg1 --steps 3 --warmup 1 > "$OUT/cfg1.json" 2> "$OUT/cfg1.err"
s=$?; echo "cfg1 exit $s"; cat "$OUT/cfg1.json"
[ $s -eq 0 ] || [ $s -eq 3 ] || exit $s
timeout -k 10 1100 python -u bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
s=$?; echo "bench exit $s"; head -c 3000 "$OUT/bench.json"; tail -5 "$OUT/bench.err"
exit $s
