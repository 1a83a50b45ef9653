# region profile (LZGPU_PROF=1 build) of the cooperative kernel: config 4 and xz
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r03l
mkdir -p $O
for c in cfg4 xz; do
  LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 \
    --no-cpu-baseline > $O/prof_$c.json 2> $O/prof_$c.err
  s=$?; echo "$c exit $s"; grep PROF $O/prof_$c.err | cut -c1-900; [ $s -eq 0 ] || exit $s
done
