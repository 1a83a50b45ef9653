# Round 5 GPU call 21: wave-uniform branches in the whole symbol loop
# (LZGPU_UNI_IF=2, the default build) against NORMALIZE only (uni1) and none
# (nouni) on configs 2, 5, 4 and the xz leg, two rounds; parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run21
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/liblzmagpu_nouni.so $V/liblzmagpu_uni1.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 600 \
  --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest.log)"; [ $s -eq 0 ] || exit $s
run() {  # cfg tag lib
  local c=$1 t=$2 L=$3
  LZGPU_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/${c}_$t.json 2>> $O/ab.err || return $?
  echo "$c $t: $(python -c "import json;d=json.load(open('$O/${c}_$t.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for r in 1 2; do
  for c in cfg2 cfg5 cfg4 xz; do
    run $c uni2_r$r "" || exit $?
    run $c uni1_r$r $V/liblzmagpu_uni1.so || exit $?
    run $c nouni_r$r $V/liblzmagpu_nouni.so || exit $?
  done
done
