#!/bin/bash
# Parity tests then a short bench (no CPU leg); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f ms/step %.4f kern_us %.1f frac %.3f single %.0f rmse %.4f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_us'], d['roofline']['frac'], d['single_chain_steps_per_s'] or 0, d['test_rmse']))"
exit $rc
