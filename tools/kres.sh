#!/bin/bash
# Register / spill / LDS metadata of the kernels in a built object: bash tools/kres.sh <obj.o> [name regex]
set -e
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --input=$T/fb --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/dev.o --unbundle
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/dev.o | python3 -c "
import sys, re
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else '.')
cur = {}
out = []
for line in sys.stdin:
    m = re.match(r'\s+\.(\w+):\s+(.*)', line)
    if not m: continue
    k, v = m.groups()
    if k in ('agpr_count','vgpr_count','vgpr_spill_count','sgpr_spill_count','group_segment_fixed_size','name','private_segment_fixed_size'):
        cur[k] = v
    if k == 'name' and 'vgpr_count' in cur:
        pass
    if k == 'wavefront_size':
        if pat.search(cur.get('name','')):
            print(cur.get('vgpr_count'), cur.get('agpr_count'), 'spill', cur.get('vgpr_spill_count'), 'priv', cur.get('private_segment_fixed_size'), cur.get('name','')[:110])
        cur = {}
" "${2:-.}"
rm -rf $T
