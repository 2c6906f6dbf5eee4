#!/bin/bash
# PMC counter passes of the chain step kernel (kernel-trace only, one group per pass; never
# combined with sys/runtime traces), summarised by scripts/pmc_chain_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_chain_${TAG:-x}
mkdir -p $OUT
ARGS="--engine chain --steps 200 --warmup 50 --epochs 1 --no-single-chain --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_chain_summary.py $OUT
