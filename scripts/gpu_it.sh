#!/bin/bash
# Iteration check: the -m gpu suite (or KSEL subset), 256-chain phase stamps of the chain engine,
# one driver-shaped bench line (--steps 20 --warmup 5) and one long bench line.  Stops at the
# first failure.  TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-it}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} \
  > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAILED|Error|error" gpurun_out/t_$TAG.log | head -20; tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
GPTSGLD_LIB=${STAMP_LIB:-gpt_amd/libgptsgld.so} timeout -k 10 200 python -u scripts/phase_stamps.py --engine chain --chains 256 > gpurun_out/stamps_$TAG.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_$TAG.txt
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print('%s: value %.0f ms/step %.4f kernel_us %.1f frac %.3f single %s' % (sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d['roofline']['frac'], d['single_chain'] and '%.0f (%s %.1f us)' % (d['single_chain']['steps_per_s'], d['single_chain']['engine'], d['single_chain']['kernel_us'])))" "$1" "$2"; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --epochs 1 --no-cpu-baseline > gpurun_out/bench20_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench20_$TAG.log; exit 1; }
summ gpurun_out/bench20_$TAG.log driver-form
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 200 --epochs 1 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
summ gpurun_out/bench_$TAG.log long
