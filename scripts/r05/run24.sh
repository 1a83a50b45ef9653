# Round 5 GPU call 24: the fast tail (the last < 20 input bytes of a one-shot
# decode in one bulk pass, checked afterwards, exact retry on a truncated
# stream): per-kernel parity and a 20k fuzz through every instantiation, then
# A/B against LZGPU_FAST_TAIL=0 on config 3 (two rounds) and configs 2, 5, 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run24
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/liblzmagpu_nofast.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_dropin_mirror.py -x -q --timeout 600 \
  --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest.log)"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ_CASES=20000 LZGPU_FUZZ_SEED=24 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q \
  --timeout 500 --timeout-method thread -k "test_fuzz_vs_oracle_each_kernel" > $O/fuzz_20k.log 2>&1
s=$?; echo "fuzz 20k exit $s: $(tail -1 $O/fuzz_20k.log)"; [ $s -eq 0 ] || exit $s
run() {  # cfg tag lib
  local c=$1 t=$2 L=$3
  LZGPU_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/${c}_$t.json 2>> $O/ab.err || return $?
  echo "$c $t: $(python -c "import json;d=json.load(open('$O/${c}_$t.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for r in 1 2; do
  run cfg3 fast_r$r "" || exit $?
  run cfg3 nofast_r$r $V/liblzmagpu_nofast.so || exit $?
done
for c in cfg2 cfg5 cfg4; do
  run $c fast_r1 "" || exit $?
  run $c nofast_r1 $V/liblzmagpu_nofast.so || exit $?
done
