#!/bin/bash
# GEMM wave-tile comparison for the stacked-sample prediction, then a rocprof kernel-trace of it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/time_pred.py ${TP_ARGS:-} > gpurun_out/time_pred.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/time_pred.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tstats -o run -- python3 scripts/time_pred.py --reps 1 ${TP_ARGS:-} > gpurun_out/tstats.log 2>&1
rc=$?; echo "rocprof rc=$rc"; cut -c1-160 gpurun_out/tstats/run_kernel_stats.csv | head -8
