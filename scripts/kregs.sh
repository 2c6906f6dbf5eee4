#!/bin/bash
# Per-kernel VGPR / spill report of one HIP source (gfx950), e.g. scripts/kregs.sh gpt_amd/csrc/chain.hip
src=$(readlink -f "$1"); shift
d=$(mktemp -d)
cd "$d" && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics "$@" --save-temps=obj -c "$src" -o x.o 2>&1 | grep -E "error" 
python3 - "$d" <<'PY'
import re, sys, glob
s = open(glob.glob(sys.argv[1] + '/*gfx950.s')[0]).read()
for blk in re.findall(r'- \.agpr_count:.*?\.wavefront_size', s, re.S):
    d = dict(re.findall(r'\.(\w+):\s+(\S+)', blk))
    print('%-60s vgpr %3s agpr %3s spill %4s priv %5s lds %s' % (d.get('name','')[:60], d.get('vgpr_count'), d.get('agpr_count'), d.get('vgpr_spill_count'), d.get('private_segment_fixed_size'), d.get('group_segment_fixed_size')))
PY
rm -rf "$d"
