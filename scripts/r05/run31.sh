# Round 5 GPU call 31: config 5's sensitivity to workgroups per CU (the merged
# latency class runs 15: its widest slices, lc+lp = 4 at pb = 4, keep 16 from
# fitting) -- 15 / 14 / 12, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run31
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
run() {  # tag env...
  local t=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/cfg5_$t.json 2>> $O/ab.err || return $?
  echo "cfg5 $t: $(python -c "import json;d=json.load(open('$O/cfg5_$t.json'));print(d['value'], d['ms_per_step'], d['verified'], d['config']['kernel_plan'])")"
}
for r in 1 2; do
  run g15_r$r X=1 || exit $?
  run g14_r$r LZGPU_GROUPS=14 || exit $?
  run g12_r$r LZGPU_GROUPS=12 || exit $?
done
