#!/bin/bash
# Round-2 GPU check: the whole -m gpu suite, then one driver-shaped bench line.  Stops at the
# first failure (no GPU step after a failed one).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r2a}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 \
  || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
