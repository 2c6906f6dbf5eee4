#!/bin/bash
# Chain-kernel library variants (gpt_amd/libgptsgld_<v>.so; "base" = gpt_amd/libgptsgld.so):
# 256-chain phase stamps + short bench each.  ENVX is passed to every run.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  lib=gpt_amd/libgptsgld_$v.so; [ "$v" = base ] && lib=gpt_amd/libgptsgld.so
  echo "=== $v"
  env $ENVX GPTSGLD_LIB=$lib timeout -k 10 120 python scripts/phase_stamps.py --engine chain --chains 256 --steps 20 > gpurun_out/var_$v.log 2>&1 || { echo "stamps $v failed rc=$?"; tail -5 gpurun_out/var_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/var_$v.log | tail -14
  env $ENVX GPTSGLD_LIB=$lib timeout -k 10 150 python bench.py --engine chain --steps 600 --warmup 100 --epochs 1 --no-single-chain --no-cpu-baseline > gpurun_out/varbench_$v.log 2>&1 || { echo "bench $v failed rc=$?"; tail -5 gpurun_out/varbench_$v.log; exit 1; }
  tail -1 gpurun_out/varbench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench value %.0f kern_us %.1f frac %.3f' % (d['value'], d['roofline']['kernel_us'], d['roofline']['frac']))"
done
