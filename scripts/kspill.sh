#!/bin/bash
# Per-kernel VGPR / spill report (gfx950) of one HIP source, keeping the .s in $OUTDIR (default /tmp/isa).
src=$(readlink -f "$1"); shift
d=${OUTDIR:-/tmp/isa}; mkdir -p "$d"; rm -f "$d"/*.s
cd "$d" && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -DGPT_NT=512 -DGPT_WPE=2 "$@" --save-temps=obj -c "$src" -o x.o 2>&1 | grep -E "error" | head
python3 - "$d" <<'PY'
import re, sys, glob
s = open(glob.glob(sys.argv[1] + '/*gfx950.s')[0]).read()
for blk in re.findall(r'- \.agpr_count:.*?\.wavefront_size', s, re.S):
    d = dict(re.findall(r'\.(\w+):\s+(\S+)', blk))
    print('%-52s vgpr %3s vspill %4s sspill %4s priv %5s' % (d.get('name','')[:52], d.get('vgpr_count'), d.get('vgpr_spill_count'), d.get('sgpr_spill_count'), d.get('private_segment_fixed_size')))
PY
