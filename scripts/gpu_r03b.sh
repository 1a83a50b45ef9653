# round-3 batch: GPU suite, strong-scaling shares, write attribution
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03b}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
s=$?; echo "pytest exit $s"; tail -4 "$OUT/pytest_gpu.log"
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
bash scripts/gpu_points.sh "${1:-r03b}_shares" cfg3:: cfg3:32768: cfg3:16384: cfg3:8192: cfg3:4096: cfg3:8192:LZGPU_THR_FIT=0 cfg2:: cfg2:2048: cfg2:1024: cfg2:512: cfg5:: || exit $?
bash scripts/attrib_shadow.sh "${1:-r03b}" > "$OUT/attrib.log" 2>&1
s=$?; echo "attrib exit $s"; tail -3 "$OUT/attrib.log"
exit $s
