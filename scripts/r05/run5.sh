# Round 5 GPU call 5: the SIMD issue micro-benchmark with per-wave occupancy
# and clock records (are W waves per SIMD co-resident, at which shader clock;
# VERDICT r04 item 1), and config-3 / config-2 region profiles with the input-
# tail and table-init counters (item 6).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run5
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
timeout -k 10 300 ./scripts/ubench/simd_issue_ubench > $O/simd_issue.jsonl 2> $O/simd_issue.err
s=$?; echo "ubench exit $s: $(grep occupancy $O/simd_issue.jsonl | tr '\n' ' ' | cut -c1-1500)"; [ $s -eq 0 ] || exit $s
for c in cfg3 cfg2; do
  LZGPU_LIB=$V/liblzmagpu_prof2.so timeout -k 10 300 python -u bench.py --config $c --steps 1 --warmup 1 \
    --no-cpu-baseline --no-e2e --no-crc --no-secondary > $O/prof_$c.json 2> $O/prof_$c.err
  s=$?; echo "prof $c exit $s: $(grep PROF $O/prof_$c.err | cut -c1-1600)"; [ $s -eq 0 ] || exit $s
done
