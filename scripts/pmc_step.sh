#!/bin/bash
# PMC counters of sgld_step_kernel (separate passes, kernel-trace only; never with sys-trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
OUT=gpurun_out/pmc
ARGS="--chains ${CHAINS:-28} --steps 400 --warmup 200 --no-cpu-baseline --kernel-steps 20"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($PMC) failed"; tail -5 $OUT/p$i.log; }
done
echo done
