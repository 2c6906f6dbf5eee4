#!/bin/bash
# Round-3b iteration: parity suite, clock-independent cycles of chain-kernel variants, single-chain
# sweep, short bench line.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${PYT:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3b_parity.log 2>&1 || { echo "parity failed"; grep -E "FAILED|Error|assert" gpurun_out/r3b_parity.log | head -20; tail -20 gpurun_out/r3b_parity.log; exit 1; }
tail -1 gpurun_out/r3b_parity.log
timeout -k 10 400 python -u scripts/ablation_run.py ${ABL:-old base} > gpurun_out/r3b_ablation.txt 2>&1 || { echo "ablation failed"; tail -20 gpurun_out/r3b_ablation.txt; exit 1; }
cat gpurun_out/r3b_ablation.txt
timeout -k 10 200 python -u scripts/single_chain.py --splits 0,2 --steps 3000 --warmup 300 > gpurun_out/r3b_single.txt 2>&1 || { echo "single failed"; tail -20 gpurun_out/r3b_single.txt; exit 1; }
grep "{" gpurun_out/r3b_single.txt
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/r3b_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r3b_bench.log; exit 1; }
tail -1 gpurun_out/r3b_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f kernel_us %.1f frac %.3f single %.0f (%s %.1f us) pred %s' % (d['value'], d['roofline']['kernel_us'], d['roofline']['frac'], d['single_chain']['steps_per_s'], d['single_chain']['engine'], d['single_chain']['kernel_us'], d.get('pred',{}).get('ms')))"
