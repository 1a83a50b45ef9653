# kernel resource usage (VGPRs, private segment, spills) of an object's gfx950 code
# usage: kres.sh obj.o [name-filter]
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$1" || exit 1
$B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/fb.bin --output=$T/k.co --unbundle || exit 1
$B/llvm-readelf --notes $T/k.co | python3 -c "
import sys,re
f=sys.argv[1]
t=sys.stdin.read()
for blk in t.split('.agpr_count')[1:]:
  m=re.search(r'\.name:\s+(\S+)',blk)
  if not m or f not in m.group(1): continue
  g=lambda k: re.search(r'\.'+k+r':\s+(\d+)',blk).group(1)
  print(m.group(1)[:80],'vgpr',g('vgpr_count'),'priv',g('private_segment_fixed_size'),'spill',g('vgpr_spill_count'))
" "${2:-lds_kernel}"
rm -rf $T
