# round-3: GPU suite on the current build, then cooperative-kernel A/B (variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03c}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
s=$?; echo "pytest exit $s"; grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -5; tail -2 "$OUT/pytest_gpu.log"
[ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
V=lzma-sdk-zliblike_amd/lib/variants
pts=()
for rep in 1 2; do
  for v in base neither nobatch nomlit; do
    pts+=("cfg4::LZGPU_LIB=$GRAFT_REPO_ROOT/$V/liblzmagpu_$v.so")
    pts+=("cfg1::LZGPU_LIB=$GRAFT_REPO_ROOT/$V/liblzmagpu_$v.so")
  done
done
bash scripts/gpu_points.sh "${1:-r03c}_ab" "${pts[@]}"
