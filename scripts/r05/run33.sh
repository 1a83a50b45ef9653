# Round 5 GPU call 33: the slot-global latency placement (kLdsMaskLatSlotG)
# where the widest slice costs workgroups per CU -- the kernel and parity
# suites, then config 5 with it (16 per CU) and without (LZGPU_SLOTG=0: 14),
# two rounds, configs 2 and 3 unchanged.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run33
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_sliced.py -x -q \
  --timeout 600 --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest.log)"; [ $s -eq 0 ] || exit $s
run() {  # cfg tag env...
  local c=$1 t=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/${c}_$t.json 2>> $O/ab.err || return $?
  echo "$c $t: $(python -c "import json;d=json.load(open('$O/${c}_$t.json'));print(d['value'], d['ms_per_step'], d['verified'], d['config'].get('kernel_plan'))" | cut -c1-300)"
}
for r in 1 2; do
  run cfg5 slotg_r$r X=1 || exit $?
  run cfg5 lds_r$r LZGPU_SLOTG=0 || exit $?
done
run cfg2 default X=1 || exit $?
run cfg3 default X=1 || exit $?
