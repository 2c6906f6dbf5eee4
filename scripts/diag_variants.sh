#!/bin/bash
# Chain-engine phase stamps for diagnostic library variants (gpt_amd/libgptsgld_<v>.so built with
# EXTRA=-DCHAIN_EXP_NOSTAGE=1 etc.; "base" = the product library), 256 chains.
cd "${GRAFT_REPO_ROOT}"
for v in base nostage nov; do
  lib=gpt_amd/libgptsgld_$v.so; [ "$v" = base ] && lib=gpt_amd/libgptsgld.so
  echo "=== $v"
  GPTSGLD_LIB=$lib timeout -k 10 120 python scripts/phase_stamps.py --engine chain --chains 256 --steps 10 > gpurun_out/d_$v.log 2>&1 || { echo fail; tail -3 gpurun_out/d_$v.log; exit 1; }
  grep -v amdgpu gpurun_out/d_$v.log | head -12
done
