#!/bin/bash
# Chains-per-GPU sweep of bench.py (one process at a time; stops at the first failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for C in ${CHAINS:-1 9 28 56 112}; do
  timeout -k 10 200 python bench.py --chains $C --steps ${STEPS:-1000} --warmup 200 --no-cpu-baseline \
      > gpurun_out/sweep_C$C.log 2>&1 || { echo "C=$C failed rc=$?"; tail -5 gpurun_out/sweep_C$C.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_C$C.log').read().strip().splitlines()[-1]); print('C=%d value=%.0f ms/step=%.4f kern_us=%.2f frac=%.3f rmse=%.4f' % ($C, d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d['roofline']['frac'], d['test_rmse']))"
done
