#!/bin/bash
# Chain-engine ablation libraries (CPU side, cross-compiled): chain.hip with entry / exit stamps
# only (CHAIN_TIMELINE=2, the product default: no stamp code in the step loop), one experiment
# flag each, linked with the other objects
# of `make timeline`.  Results are wrong by construction; scripts/ablation_run.py measures their
# shader-clock cycles per step on the GPU (clock-independent).
#   scripts/ablation_build.sh base "" nonoise -DCHAIN_EXP_NONOISE=1 ...
set -e
cd "$(dirname "$0")/../gpt_amd/csrc"
make -s timeline
FLAGS="-DGPT_NT=512 -DGPT_WPE=2 --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics"
mkdir -p build_abl
others=$(ls build_tl/*.o | grep -v chain.o)
pids=()
while [ $# -gt 0 ]; do
  name=$1; extra=$2; shift 2
  ( /opt/rocm/bin/hipcc $FLAGS $extra -c chain.hip -o build_abl/chain_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others build_abl/chain_$name.o \
      -o ../libgptsgld_abl_$name.so && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
