#!/bin/bash
# Test-RMSE runs of kin40kExperiment.jl's configuration (scripts/kin40k_experiment.py); each run
# has its own time limit and the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { tag=$1; shift
  timeout -k 10 300 python scripts/kin40k_experiment.py --out gpurun_out/kin40k_$tag.npz "$@" > gpurun_out/kin40k_$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/kin40k_$tag.log; [ $rc -eq 0 ] || exit $rc; }
run ref
run fixed --fixed
run ref_eps5 --epsw 1e-5 --epsU 1e-8
