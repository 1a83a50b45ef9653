# wave64 cooperative A/B + cfg1 leg with the 64 MiB-dic loop
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=lzma-sdk-zliblike_amd/lib/variants
pts=()
for rep in 1 2; do
  for v in base w64; do
    pts+=("cfg4::LZGPU_LIB=$GRAFT_REPO_ROOT/$V/liblzmagpu_$v.so")
    pts+=("xz::LZGPU_LIB=$GRAFT_REPO_ROOT/$V/liblzmagpu_$v.so")
  done
done
bash scripts/gpu_points.sh "${1:-r03d}_ab" "${pts[@]}" || exit $?
mkdir -p gpurun_out/${1:-r03d}
timeout -k 10 300 python -u bench.py --config cfg1 --steps 3 --warmup 1 > gpurun_out/${1:-r03d}/cfg1.json 2> gpurun_out/${1:-r03d}/cfg1.err
s=$?; echo "cfg1 exit $s"; cat gpurun_out/${1:-r03d}/cfg1.json | head -c 2500; exit $s
