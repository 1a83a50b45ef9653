# Round 5 GPU call 2: SIMD issue micro-benchmark; GPU
# parity of the pruned build + the one-lane LDS window (item 2: per-kernel
# matrix, full configs 2/3/5); config 2 / 5 A/B of the window (off / write-
# through / deferred) over two rounds; region profiles (LZGPU_PROF=1 variant)
# of configs 2 (window on and off), 5 and 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run2
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
timeout -k 10 240 ./scripts/ubench/simd_issue_ubench > $O/simd_issue.jsonl 2> $O/simd_issue.err
s=$?; echo "ubench exit $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread \
  -m gpu > $O/pytest_kernels.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest_kernels.log)"; [ $s -eq 0 ] || exit $s
for round in 1 2; do
  for v in win off wt; do
    E=""; L=""
    [ $v = off ] && E="LZGPU_LANE_WIN=0"
    [ $v = wt ] && L=$V/liblzmagpu_wt.so
    for c in cfg2 cfg5; do
      env $E LZGPU_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 \
        --no-cpu-baseline --no-e2e --no-crc --no-secondary > $O/${c}_${v}_r$round.json 2>> $O/ab.err
      s=$?; echo "$c $v r$round exit $s: $(python -c "import json;d=json.load(open('$O/${c}_${v}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])" 2>&1)"
      [ $s -eq 0 ] || exit $s
    done
  done
done
for t in cfg2:win cfg2:off cfg5:win cfg3:win; do
  c=${t%%:*}; v=${t#*:}; E=""; [ $v = off ] && E="LZGPU_LANE_WIN=0"
  env $E LZGPU_LIB=$V/liblzmagpu_prof.so timeout -k 10 300 python -u bench.py --config $c --steps 1 --warmup 1 \
    --no-cpu-baseline --no-e2e --no-crc --no-secondary > $O/prof_${c}_$v.json 2> $O/prof_${c}_$v.err
  s=$?; echo "prof $c $v exit $s: $(grep PROF $O/prof_${c}_$v.err | cut -c1-1500)"; [ $s -eq 0 ] || exit $s
done
