# cooperative LZ copy (lz_copy_coop): GPU suite on the new library, then A/B
# against the HEAD build (lib/variants/liblzmagpu_base.so) on configs 4, xz, 1;
# then the region profile of the HEAD build (LZGPU_PROF=1) on config 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -4 $O/pytest_gpu.log; [ $s -eq 0 ] || exit $s
pts=()
for rep in 1 2; do
  pts+=("cfg4::LZGPU_LIB=$V/liblzmagpu_base.so" "cfg4::" "xz::LZGPU_LIB=$V/liblzmagpu_base.so" "xz::")
done
bash scripts/gpu_points.sh r03m/ab "${pts[@]}" || exit $?
for v in base new; do
  e=""; [ $v = base ] && e="LZGPU_LIB=$V/liblzmagpu_base.so"
  env $e timeout -k 10 300 python -u bench.py --config cfg1 --steps 3 --warmup 1 > $O/cfg1_$v.json 2> $O/cfg1_$v.err
  s=$?; echo "cfg1 $v exit $s"; cut -c1-300 $O/cfg1_$v.json; [ $s -eq 0 ] || exit $s
done
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/prof_cfg4.json 2> $O/prof_cfg4.err
s=$?; echo "prof exit $s"; grep PROF $O/prof_cfg4.err | cut -c1-1200
exit $s
