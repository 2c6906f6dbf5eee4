#!/bin/bash
# Prediction-path check: GPU parity tests, a bench run, a rocprofv3 kernel-trace of the bench
# (per-kernel stats incl. the MFMA GEMM), and the same prediction through the per-sample
# streaming kernel (GPTSGLD_PRED=direct) for comparison.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f kern_us %.1f rmse %.4f pred %s' % (d['value'], d['roofline']['kernel_us'], d['test_rmse'], d['pred']))"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pstats -o run -- python3 bench.py --steps 500 --warmup 100 --no-cpu-baseline --no-single-chain > gpurun_out/pstats.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cut -c1-150 gpurun_out/pstats/run_kernel_stats.csv | head -6
[ "${DIRECT:-0}" = 1 ] || exit 0
GPTSGLD_PRED=direct timeout -k 10 200 python bench.py --steps 200 --warmup 50 --no-cpu-baseline --no-single-chain > gpurun_out/bench_direct.log 2>&1
rc=$?; echo "direct rc=$rc"; tail -1 gpurun_out/bench_direct.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('direct pred ms %.2f rmse %.6f' % (d['pred']['ms'], d['test_rmse']))"
exit $rc
