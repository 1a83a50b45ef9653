# cooperative length-coder choice speculation A/B: parity
# of the variant on the cooperative kernel, then cfg4 / xz / cfg1 alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
mkdir -p gpurun_out/r03h
LZGPU_LIB=$V/liblzmagpu_lenspec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q \
  --timeout 300 --timeout-method thread -k "coop" > gpurun_out/r03h/pytest_lenspec.log 2>&1
s=$?; tail -3 gpurun_out/r03h/pytest_lenspec.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2; do
  for v in base lenspec; do
    pts+=("cfg4::LZGPU_LIB=$V/liblzmagpu_$v.so")
  done
done
for v in base lenspec; do pts+=("xz::LZGPU_LIB=$V/liblzmagpu_$v.so" "cfg1::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
bash scripts/gpu_points.sh r03h_ab "${pts[@]}"
