# Round 5 GPU call 39 (prepared, not run this round): length coders loaded
# ahead of the literal batch (variant LZGPU_LEN_PF=1, throughput kernel, pb = 0)
# vs loaded at the match (default); configs 3 / 4 bench A/B in two rounds, then
# the variant's GPU parity suite.  Build first:
#   make -C lzma-sdk-zliblike_amd variants VARIANT_SET="lenpf:LZGPU_LEN_PF=1"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run39
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/liblzmagpu_lenpf.so > $O/binary.sha256
run() {  # cfg tag lib
  local c=$1 t=$2 L=$3
  LZGPU_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary > $O/${c}_$t.json 2>> $O/ab.err || return $?
  echo "$c $t: $(python -c "import json;d=json.load(open('$O/${c}_$t.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for r in 1 2; do
  run cfg3 base_r$r "" || exit $?
  run cfg3 lenpf_r$r $V/liblzmagpu_lenpf.so || exit $?
done
run cfg4 base "" || exit $?
run cfg4 lenpf $V/liblzmagpu_lenpf.so || exit $?
LZGPU_LIB=$V/liblzmagpu_lenpf.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1
s=$?; echo "gpu suite exit $s: $(tail -1 $O/gpu_suite.log)"; exit $s
