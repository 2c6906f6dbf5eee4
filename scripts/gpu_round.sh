#!/bin/bash
# Iteration check on the GPU box: the whole -m gpu suite, 256-chain phase stamps of the chain
# engine, one short bench line.  Stops at the first failure.  TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-it}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} \
  > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAILED|Error|error" gpurun_out/t_$TAG.log | head -20; tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 200 python -u scripts/phase_stamps.py --engine chain --chains 256 > gpurun_out/stamps_$TAG.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_$TAG.txt
timeout -k 10 300 python -u bench.py --steps 400 --warmup 50 --epochs 1 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f kernel_us %.1f frac %.3f single %.0f (%s %.1f us)' % (d['value'], d['roofline']['kernel_us'], d['roofline']['frac'], d['single_chain']['steps_per_s'], d['single_chain']['engine'], d['single_chain']['kernel_us']))"
