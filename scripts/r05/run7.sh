# Round 5 GPU call 7: (a) the SIMD issue micro-benchmark over the number of
# active lanes per wave (a lone one-lane wave issued a VALU instruction per ~16
# cycles); (b) the latency kernel's stream run by D lanes of one wave
# (LZGPU_DUP=D: lzgpu_decode_dup_kernel) -- per-kernel parity, then config 2
# and config 5 A/B; (c) the config-3 wave-shape experiment (run6.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run7
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 300 ./scripts/ubench/simd_issue_ubench lanes > $O/simd_lanes.jsonl 2> $O/simd_lanes.err
s=$?; echo "ubench lanes exit $s"; [ $s -eq 0 ] || exit $s
for D in 2 32; do
  LZGPU_DUP=$D timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 \
    --timeout-method thread -m gpu -k "latency or cfg2 or cfg5" > $O/pytest_dup$D.log 2>&1
  s=$?; echo "pytest dup $D exit $s: $(tail -1 $O/pytest_dup$D.log)"; [ $s -eq 0 ] || exit $s
done
for r in 1 2; do
  for D in 0 2 4 32; do
    LZGPU_DUP=$D timeout -k 10 300 python bench.py --config cfg2 --steps 5 --warmup 1 --no-cpu-baseline \
      --no-e2e --no-crc --no-secondary > $O/cfg2_dup${D}_r$r.json 2>> $O/ab.err || exit $?
    echo "cfg2 dup $D r$r: $(python -c "import json;d=json.load(open('$O/cfg2_dup${D}_r$r.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
  done
done
for D in 0 2 32; do
  LZGPU_DUP=$D timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/cfg5_dup$D.json 2>> $O/ab.err || exit $?
  echo "cfg5 dup $D: $(python -c "import json;d=json.load(open('$O/cfg5_dup$D.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
done
bash scripts/r05/run6.sh
