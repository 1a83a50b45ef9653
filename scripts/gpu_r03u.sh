# region profile (LZGPU_PROF=1 build of the round-3 HEAD source) of the
# cooperative kernel on config 4 and of the single-stream config 1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r03u
mkdir -p $O
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/prof_cfg4.json 2> $O/prof_cfg4.err
s=$?; echo "cfg4 exit $s"; grep PROF $O/prof_cfg4.err | cut -c1-1500; [ $s -eq 0 ] || exit $s
