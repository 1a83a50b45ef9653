# branch-free checkpoint reader A/B (LZGPU_RDQ_UNCOND): parity of the variant on
# the throughput and cooperative kernels, then cfg3 / cfg4 / xz alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
mkdir -p gpurun_out/r03j
LZGPU_LIB=$V/liblzmagpu_rdq.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q \
  --timeout 300 --timeout-method thread -k "throughput or coop" > gpurun_out/r03j/pytest_rdq.log 2>&1
s=$?; tail -3 gpurun_out/r03j/pytest_rdq.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2; do
  for v in base rdq; do
    pts+=("cfg3::LZGPU_LIB=$V/liblzmagpu_$v.so" "cfg4::LZGPU_LIB=$V/liblzmagpu_$v.so")
  done
done
for v in base rdq; do pts+=("xz::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
bash scripts/gpu_points.sh r03j_ab "${pts[@]}"
