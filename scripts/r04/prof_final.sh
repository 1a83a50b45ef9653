# Round 4: region profile (LZGPU_PROF=1 build of the final source) of the
# cooperative kernel on config 4 -- where its cycles go after the round-4
# changes (serial literal tree, window, deferred output, direct-bit runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_regions
mkdir -p $O
LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-gather > $O/prof_cfg4.json 2> $O/prof_cfg4.err || exit $?
echo "cfg4: $(grep PROF $O/prof_cfg4.err | cut -c1-1500)"
