# literal batch per pass for the one-lane latency waves (configs 2 and 5, 7z):
# LZGPU_LIT_BATCH 1 / 3 (first pass: -14 % / -2 % on config 2) and 16 / 64 against HEAD's 8 (a one-lane wave has no neighbours
# to wait for, so the batch loop is pure overhead there)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/lzma-sdk-zliblike_amd/lib/variants
pts=()
for rep in 1 2; do
  for v in head lb16 lb64; do pts+=("cfg2::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
done
for v in head lb16 lb64; do pts+=("cfg5::LZGPU_LIB=$V/liblzmagpu_$v.so"); done
bash scripts/gpu_points.sh r03s/ab "${pts[@]}"
