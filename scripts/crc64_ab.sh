# A/B of CRC-64 code shapes on the xz leg (run via gpurun): main vs lib/variants builds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
for v in ${VARIANTS:-main x2 x8}; do
  if [ $v = main ]; then lib=$PWD/lzma-sdk-zliblike_amd/lib/liblzmagpu.so; else lib=$PWD/lzma-sdk-zliblike_amd/lib/variants/liblzmagpu_$v.so; fi
  LZGPU_LIB=$lib timeout -k 10 300 python bench.py --config xz --steps 5 --warmup 1 > gpurun_out/crc64_${v}_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/crc64_${v}_$r.json'));k=d['config']['kernel_ms'];print('$v r$r', k, d.get('crc64') or d['config'].get('crc64'), d['verified'])"
done
done
