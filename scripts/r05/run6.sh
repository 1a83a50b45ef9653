# Round 5 GPU call 6: config-3 wave shape with more waves
# per SIMD.  Variant t3: IsRep/G0/G1/G2 moved from LDS to the global rows
# (placement 0x101: 540 B of LDS per stream instead of 636, so 288 lanes fit a
# CU) and a 3-waves-per-SIMD build; shapes: 32 x 8 (the default, W = 2),
# 24 x 12 (W = 3, all 256 streams of a CU resident), 16 x 16 (W = 4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run6
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
run() {  # tag lib env...
  local t=$1 L=$2; shift 2
  env "$@" LZGPU_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    --no-crc --no-secondary > $O/cfg3_$t.json 2>> $O/ab.err || return $?
  echo "cfg3 $t: $(python -c "import json;d=json.load(open('$O/cfg3_$t.json'));k=d['config']['kernel_plan'];print(d['value'], d['ms_per_step'], d['verified'], k['streams_per_workgroup'], k['workgroups_per_cu'], k['waves_per_simd'], k['placement'])")"
}
T=$V/liblzmagpu_t3.so
for r in 1 2; do
  run base_r$r "" X=1 || exit $?
  run t3_w2_r$r $T X=1 || exit $?
  run t3_w3ilv_r$r $T LZGPU_LANES=24 LZGPU_GROUPS=12 LZGPU_OCC=3 LZGPU_ILV_ANY=1 || exit $?
  run t3_w3sl_r$r $T LZGPU_LANES=24 LZGPU_GROUPS=12 LZGPU_OCC=3 LZGPU_ILV=0 || exit $?
  run t3_w4ilv_r$r $T LZGPU_LANES=16 LZGPU_GROUPS=16 LZGPU_OCC=4 LZGPU_ILV_ANY=1 || exit $?
done
