#!/bin/bash
# Grid-engine (sgld.hip) experiment libraries: sgld.hip rebuilt with one set of -D flags each,
# linked with the product's other objects.  scripts/phase_stamps.py with GPTSGLD_LIB pointing at
# one of them measures its per-phase shader cycles on the GPU.
#   scripts/sgld_variants.sh notouch -DGPT_TOUCH=0 tile -DVPHASE_COLS=0 ...
set -e
cd "$(dirname "$0")/../gpt_amd/csrc"
make -s
FLAGS="-DGPT_NT=512 -DGPT_WPE=2 --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics"
mkdir -p build_sv
others=$(ls build/*.o | grep -v sgld.o)
pids=()
while [ $# -gt 0 ]; do
  name=$1; extra=$2; shift 2
  ( /opt/rocm/bin/hipcc $FLAGS $extra -c sgld.hip -o build_sv/sgld_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others build_sv/sgld_$name.o \
      -o ../libgptsgld_sv_$name.so && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
