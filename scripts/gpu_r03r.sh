# Round-3 fuzz campaigns on the shipped binary after the cooperative-kernel
# changes (cooperative copy, uniform stage stores): 20,000 seeded LZMA streams
# and 5,000 LZMA2 items through every kernel instantiation against the oracle,
# then 200,000 LZMA streams through the two cooperative instantiations
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03r
mkdir -p $O
LZGPU_FUZZ_CASES=20000 LZGPU_FUZZ_SEED=20261017 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 500 --timeout-method thread -k "test_fuzz_vs_oracle_each_kernel" \
  > $O/fuzz_20k_seed20261017.log 2>&1
s=$?; echo "fuzz 20k exit $s"; tail -1 $O/fuzz_20k_seed20261017.log; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ2_CASES=5000 LZGPU_FUZZ2_SEED=20261017 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 500 --timeout-method thread -k "test_lzma2_fuzz_vs_oracle_each_kernel" \
  > $O/lzma2_fuzz_5k_seed20261017.log 2>&1
s=$?; echo "lzma2 fuzz 5k exit $s"; tail -1 $O/lzma2_fuzz_5k_seed20261017.log; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ_CASES=200000 LZGPU_FUZZ_SEED=1017 timeout -k 10 700 python -u -m pytest \
  tests/test_gpu_kernels.py -m gpu -v --timeout 650 --timeout-method thread \
  -k "test_fuzz_vs_oracle_each_kernel and coop" > $O/fuzz_200k_coop_seed1017.log 2>&1
s=$?; echo "fuzz 200k coop exit $s"; tail -1 $O/fuzz_200k_coop_seed1017.log
exit $s
