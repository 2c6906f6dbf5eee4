#!/bin/bash
# Round profile: bench line, rocprofv3 kernel-trace stats, and FETCH/WRITE PMC passes for the
# HBM traffic of sgld_step_kernel (separate passes, kernel-trace only).  Stops at the first
# failure.  Usage: TAG=r1 bash scripts/profile_round.sh [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="$@"
timeout -k 10 300 python3 bench.py $ARGS > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS --no-cpu-baseline --epochs 1 --no-single-chain > $OUT/stats.log 2>&1 || { echo "stats pass failed"; tail -5 $OUT/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS --no-cpu-baseline --epochs 1 --no-single-chain > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS --no-cpu-baseline --epochs 1 --no-single-chain > $OUT/write.log 2>&1 || { echo "write pass failed"; tail -5 $OUT/write.log; exit 1; }
echo "profile done"
cat $OUT/bench.json
