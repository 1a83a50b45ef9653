set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
for v in ${VARIANTS:-main c1k u8 c1ku8 c512u8}; do
  if [ $v = main ]; then lib=$PWD/lzma-sdk-zliblike_amd/lib/liblzmagpu.so; else lib=$PWD/lzma-sdk-zliblike_amd/lib/variants/liblzmagpu_$v.so; fi
  LZGPU_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-secondary > gpurun_out/crc_${v}_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/crc_${v}_$r.json'));c=d['crc32'];print('$v r$r', c['avg_ms'], c['roofline']['achieved'], c['roofline']['frac'], c['verified'], d['verified'])"
done
done
