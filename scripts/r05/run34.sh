# Round 5 GPU call 34: the final binary (fast tail, LDS-block planning, slot-global latency placement) -- smoke, the whole GPU
# suite, the default bench line, then fuzz campaigns: 50,000 LZMA streams and
# 10,000 LZMA2 items through every instantiation, 300,000 LZMA streams through
# every LDS instantiation (throughput, latency, cooperative).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run34
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s: $(tail -1 $O/smoke.log)"; [ $s -eq 0 ] || exit $s
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest_gpu.log)"; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python bench.py > $O/bench_line.json 2> $O/bench.err
s=$?; echo "bench exit $s: $(python -c "import json;d=json.load(open('$O/bench_line.json'));print(d['value'], d['ms_per_step'], d['verified'], {k:(v['value'],v['verified']) for k,v in d['secondary'].items()})")"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ_CASES=50000 LZGPU_FUZZ_SEED=20261021 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 500 --timeout-method thread -k "test_fuzz_vs_oracle_each_kernel" \
  > $O/fuzz_50k_seed20261021.log 2>&1
s=$?; echo "fuzz 50k exit $s: $(tail -1 $O/fuzz_50k_seed20261021.log)"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ2_CASES=10000 LZGPU_FUZZ2_SEED=20261021 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 500 --timeout-method thread -k "test_lzma2_fuzz_vs_oracle_each_kernel" \
  > $O/lzma2_fuzz_10k_seed20261021.log 2>&1
s=$?; echo "lzma2 fuzz 10k exit $s: $(tail -1 $O/lzma2_fuzz_10k_seed20261021.log)"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ_CASES=300000 LZGPU_FUZZ_SEED=1021 timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 850 --timeout-method thread \
  -k "test_fuzz_vs_oracle_each_kernel and not global" > $O/fuzz_300k_lds_seed1021.log 2>&1
s=$?; echo "fuzz 300k exit $s: $(tail -1 $O/fuzz_300k_lds_seed1021.log)"
exit $s
