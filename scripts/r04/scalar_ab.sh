# Round 4: one-lane latency waves on the scalar-register build
# (lzgpu_decode_one_kernel) -- GPU parity of the latency instantiations, then
# A/B of the share of waves on it (LZGPU_SCALAR=0..4) on configs 2 and 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_scalar
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 \
  --timeout-method thread -m gpu -k "latency" > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -2 $O/pytest.log; [ $s -eq 0 ] || exit $s
for round in 1 2; do
  qs="0 4 2 1 3"; [ $round -eq 2 ] && qs="0 4 2"
  for q in $qs; do
    for c in cfg2 cfg5; do
      LZGPU_SCALAR=$q timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 \
        --no-cpu-baseline --no-e2e --no-crc > $O/${c}_q${q}_r$round.json 2>> $O/ab.err || exit $?
      echo "$c scalar=$q r$round: $(python -c "import json;d=json.load(open('$O/${c}_q${q}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
    done
  done
done
