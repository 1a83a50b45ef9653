# Round 5 GPU call 36: streaming campaigns on the final binary -- 3,000 device
# sessions in lockstep, 1,000 concurrent drop-in DecodeToBuf loops, 30,000
# LZMA2 items through every instantiation, and the tail-truncation test.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_fuzz2
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
LZGPU_SESSION_FUZZ=3000 LZGPU_SESSION_SEED=5051 timeout -k 10 600 python -u -m pytest tests/test_sessions.py -v \
  --timeout 550 --timeout-method thread -m gpu -k fuzz_lockstep > $O/session_fuzz_3000_seed5051.log 2>&1
s=$?; echo "session fuzz exit $s: $(tail -1 $O/session_fuzz_3000_seed5051.log)"; [ $s -eq 0 ] || exit $s
LZGPU_DROPIN_FUZZ=1000 LZGPU_DROPIN_SEED=5052 timeout -k 10 600 python -u -m pytest tests/test_coalesce.py -v \
  --timeout 550 --timeout-method thread -m gpu -k decode_to_buf_loops_fuzz > $O/dropin_fuzz_1000_seed5052.log 2>&1
s=$?; echo "dropin fuzz exit $s: $(tail -1 $O/dropin_fuzz_1000_seed5052.log)"; [ $s -eq 0 ] || exit $s
LZGPU_FUZZ2_CASES=30000 LZGPU_FUZZ2_SEED=5053 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v \
  --timeout 550 --timeout-method thread -m gpu -k "test_lzma2_fuzz_vs_oracle_each_kernel" > $O/lzma2_fuzz_30k_seed5053.log 2>&1
s=$?; echo "lzma2 fuzz exit $s: $(tail -1 $O/lzma2_fuzz_30k_seed5053.log)"; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 250 --timeout-method thread -m gpu \
  -k tail_truncations > $O/tail_truncations.log 2>&1
s=$?; echo "tail exit $s: $(tail -1 $O/tail_truncations.log)"; exit $s
