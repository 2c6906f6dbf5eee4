#!/bin/bash
# r = 20 paths (40 x 40 Padé solve): GPU tests that reach them, grid-engine stamps at the
# reference's kin40k configuration and MovieLens config-5 timing, per library variant in VARIANTS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  lib=gpt_amd/libgptsgld_$v.so; [ "$v" = base ] && lib=gpt_amd/libgptsgld.so
  echo "=== $v"
  GPTSGLD_LIB=$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "r20 or reference_configuration or kin40k_ref or tgp or gmc or movielens" > gpurun_out/r20t_$v.log 2>&1 || { echo "tests $v failed"; tail -15 gpurun_out/r20t_$v.log; exit 1; }
  tail -1 gpurun_out/r20t_$v.log
  GPTSGLD_LIB=$lib timeout -k 10 200 python scripts/phase_stamps.py --engine grid --chains 1 --steps 10 --n 150 --r 20 2>&1 | grep -E "expm|total|event" 
  GPTSGLD_LIB=$lib timeout -k 10 300 python scripts/time_movielens.py --epochs 2 --r 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['workload'], 'sgd s/epoch %.4f steps/s %.0f five-fold s/epoch %.4f' % (d['sideinfo_sgd_s_per_epoch'], d['sideinfo_steps_per_s'], d['five_folds_one_launch_s_per_epoch']))" || exit 1
done
