#!/bin/bash
# 256-chain phase stamps + long bench for each library variant in VARIANTS (gpt_amd/libgptsgld_<v>.so;
# "base" = gpt_amd/libgptsgld.so); KSEL runs that pytest -k subset on each variant first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  lib=gpt_amd/libgptsgld_$v.so; [ "$v" = base ] && lib=gpt_amd/libgptsgld.so
  echo "=== $v"
  if [ -n "$KSEL" ]; then
    GPTSGLD_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KSEL" > gpurun_out/vt_$v.log 2>&1 || { echo "tests $v failed"; grep -E "FAILED|Error" gpurun_out/vt_$v.log | head; tail -15 gpurun_out/vt_$v.log; exit 1; }
    tail -1 gpurun_out/vt_$v.log
  fi
  GPTSGLD_LIB=$lib timeout -k 10 120 python scripts/phase_stamps.py --engine chain --chains 256 --steps 10 > gpurun_out/vs_$v.log 2>&1 || { echo "stamps $v failed rc=$?"; tail -5 gpurun_out/vs_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/vs_$v.log | sed -n '2,11p'
  GPTSGLD_LIB=$lib timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --epochs 1 --no-cpu-baseline --no-single-chain > gpurun_out/vb_$v.log 2>&1 || { echo "bench $v failed rc=$?"; tail -5 gpurun_out/vb_$v.log; exit 1; }
  tail -1 gpurun_out/vb_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench value %.0f ms/step %.4f kern_us %.1f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d['roofline']['frac']))"
done
