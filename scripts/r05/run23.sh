# Round 5 fuzz campaigns on the final binary (32-lane one-stream kernel,
# wave-uniform cooperative branches, resident-wave register budgets): 50,000
# seeded LZMA streams and 10,000 LZMA2 items through every kernel
# instantiation against the oracle, then 300,000 LZMA streams through the
# cooperative instantiations and 300,000 through the latency one.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_fuzz
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 300 python -u -m pytest tests/test_coalesce.py -v --timeout 240 --timeout-method thread -m gpu \
  -k oversized > $O/pytest_oversized.log 2>&1
s=$?; echo "oversized exit $s: $(tail -1 $O/pytest_oversized.log)"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ_CASES=50000 LZGPU_FUZZ_SEED=20261019 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 500 --timeout-method thread -k "test_fuzz_vs_oracle_each_kernel" \
  > $O/fuzz_50k_seed20261019.log 2>&1
s=$?; echo "fuzz 50k exit $s: $(tail -1 $O/fuzz_50k_seed20261019.log)"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ2_CASES=10000 LZGPU_FUZZ2_SEED=20261019 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 500 --timeout-method thread -k "test_lzma2_fuzz_vs_oracle_each_kernel" \
  > $O/lzma2_fuzz_10k_seed20261019.log 2>&1
s=$?; echo "lzma2 fuzz 10k exit $s: $(tail -1 $O/lzma2_fuzz_10k_seed20261019.log)"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ_CASES=300000 LZGPU_FUZZ_SEED=1019 timeout -k 10 700 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 650 --timeout-method thread \
  -k "test_fuzz_vs_oracle_each_kernel and (coop or latency)" > $O/fuzz_300k_coop_latency_seed1019.log 2>&1
s=$?; echo "fuzz 300k coop/latency exit $s: $(tail -1 $O/fuzz_300k_coop_latency_seed1019.log)"
exit $s
