#!/bin/bash
# Spill / wait report of the chain kernel's batch loop (R, J given), e.g. scripts/loopcheck.sh 5 8
R=${1:-5}; J=${2:-8}
d=$(mktemp -d); cd $d
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics $EXTRA --save-temps=obj -c /root/repo/gpt_amd/csrc/chain.hip -o x.o 2>/dev/null
F=$(ls *gfx950.s)
L0=$(grep -n "^_ZN3gpt12chain_kernelILi${R}ELi${J}ELi2E.*:" $F | head -1 | cut -d: -f1)
L1=$(awk -v s=$L0 'NR>s && /s_endpgm/ {print NR; exit}' $F)
sed -n "${L0},${L1}p" $F > k.s
B=$(grep -n "s_barrier" k.s | cut -d: -f1 | tr '\n' ' ')
echo "barriers at: $B"
set -- $B
echo "loop (bar1..bar4): scratch_ld $(awk -v a=$1 -v b=$4 'NR>a&&NR<b&&/scratch_load/' k.s | wc -l) scratch_st $(awk -v a=$1 -v b=$4 'NR>a&&NR<b&&/scratch_store/' k.s | wc -l) vmcnt_waits $(awk -v a=$1 -v b=$4 'NR>a&&NR<b&&/s_waitcnt.*vmcnt/' k.s | wc -l) writelane $(awk -v a=$1 -v b=$4 'NR>a&&NR<b&&/v_writelane/' k.s | wc -l) readlane $(awk -v a=$1 -v b=$4 'NR>a&&NR<b&&/v_readlane/' k.s | wc -l)"
echo "after loop: scratch_ld $(awk -v a=$4 'NR>a&&/scratch_load/' k.s | wc -l) scratch_st $(awk -v a=$4 'NR>a&&/scratch_store/' k.s | wc -l)"
awk -v a=$1 -v b=$4 'NR>a&&NR<b&&/s_waitcnt.*vmcnt|global_load_lds|scratch/ {print NR": "$0}' k.s | head -${3:-30}
cp k.s /tmp/chain_k.s
rm -rf $d
