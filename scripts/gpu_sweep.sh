#!/bin/bash
# Chains-per-GPU sweep of bench.py (one process at a time; stops at the first failure).
# LIB=<path to an alternative libgptsgld build> selects a variant (e.g. the 256-thread build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-}
for C in ${CHAINS:-1 9 28 56 112}; do
  GPTSGLD_LIB=${LIB:-} timeout -k 10 200 python bench.py --chains $C --steps ${STEPS:-1000} --warmup 200 --no-cpu-baseline ${ARGS:-} \
      > gpurun_out/sweep${TAG}_C$C.log 2>&1 || { echo "C=$C failed rc=$?"; tail -5 gpurun_out/sweep${TAG}_C$C.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep${TAG}_C$C.log').read().strip().splitlines()[-1]); print('${TAG} C=%d value=%.0f ms/step=%.4f kern_us=%.2f frac=%.3f rmse=%.4f' % ($C, d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d['roofline']['frac'], d['test_rmse']))"
done
