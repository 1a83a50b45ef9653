# Round 4: direct bits several per step in the cooperative kernel (direct_coop)
# -- GPU parity of the cooperative paths, A/B against the bit-serial loop
# (variant build LZGPU_DIRECT_CHUNKS=0) on configs 4 and 1 and the xz leg, and
# the config-4 region profile of both (LZGPU_PROF=1 builds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_direct
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_xz.py \
  tests/test_cfg1.py tests/test_sessions.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "coop or parity or cfg1 or session or xz or cfg4 or goldens" > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -2 $O/pytest.log; [ $s -eq 0 ] || exit $s
for round in 1 2; do
  for v in base nodc; do
    L=""; [ $v = nodc ] && L=$V/liblzmagpu_nodc.so
    LZGPU_LIB=$L timeout -k 10 300 python bench.py --config cfg4 --steps 5 --warmup 1 --no-cpu-baseline \
      --no-gather > $O/cfg4_${v}_r$round.json 2>> $O/ab.err || exit $?
    echo "cfg4 $v r$round: $(python -c "import json;d=json.load(open('$O/cfg4_${v}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
    LZGPU_LIB=$L timeout -k 10 300 python bench.py --config xz --steps 5 --warmup 1 --no-cpu-baseline \
      > $O/xz_${v}_r$round.json 2>> $O/ab.err || exit $?
    echo "xz $v r$round: $(python -c "import json;d=json.load(open('$O/xz_${v}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
  done
done
for v in prof profnodc; do
  LZGPU_LIB=$V/liblzmagpu_$v.so timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-gather > $O/prof_cfg4_$v.json 2> $O/prof_cfg4_$v.err || exit $?
  echo "prof $v: $(grep PROF $O/prof_cfg4_$v.err | cut -c1-900)"
done
