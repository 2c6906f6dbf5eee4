#!/bin/bash
# MovieLens CF timing (r = 20 and 15) and the MovieLens GPU tests for each library variant in
# VARIANTS (gpt_amd/libgptsgld_<v>.so; "base" = gpt_amd/libgptsgld.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  lib=gpt_amd/libgptsgld_$v.so; [ "$v" = base ] && lib=gpt_amd/libgptsgld.so
  echo "=== $v"
  GPTSGLD_LIB=$lib timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "movielens or cf" > gpurun_out/mt_$v.log 2>&1 || { echo "tests $v failed"; tail -15 gpurun_out/mt_$v.log; exit 1; }
  tail -1 gpurun_out/mt_$v.log
  for r in 20 15; do
    GPTSGLD_LIB=$lib timeout -k 10 300 python scripts/time_movielens.py --epochs 2 --r $r 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['workload'], 'sgd s/epoch %.4f steps/s %.0f gibbs s/sweep %.4f five-fold s/epoch %.4f' % (d['sideinfo_sgd_s_per_epoch'], d['sideinfo_steps_per_s'], d['gibbs_s_per_sweep'], d['five_folds_one_launch_s_per_epoch']))" || exit 1
  done
done
