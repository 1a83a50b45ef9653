# Round 4: lane-interleaved LDS slices in the throughput kernel (cell i of lane
# l at i * 32 + l: reads of diverging tree nodes in different banks) -- GPU
# parity of the throughput paths, A/B against per-lane slices
# (-DLZGPU_LDS_ILV=0) on config 3, and the bank-conflict counter of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
O=gpurun_out/r04_ldsilv
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_xz.py tests/test_7z.py \
  -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -1 $O/pytest.log; [ $s -eq 0 ] || exit $s
for round in 1 2; do
  for v in ilv nolds; do
    L=""; [ $v != ilv ] && L=$V/liblzmagpu_$v.so
    LZGPU_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-crc \
      > $O/cfg3_${v}_r$round.json 2>> $O/ab.err || exit $?
    echo "cfg3 $v r$round: $(python -c "import json;d=json.load(open('$O/cfg3_${v}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in ilv nolds; do
  L=""; [ $v != ilv ] && L=$V/liblzmagpu_$v.so
  LZGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES \
    -d $GRAFT_REPO_ROOT/$O/pmc_$v -o pmc --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-e2e --no-crc \
    > $GRAFT_REPO_ROOT/$O/pmc_$v.json 2> $GRAFT_REPO_ROOT/$O/pmc_$v.err || exit $?
  echo "pmc $v done"
done
