#!/bin/bash
# One GPU session of round-4 checks, each step under its own time limit; a test failure (rc 1) is
# logged and the session goes on, a time limit / abort / segfault (124, 137, 134, 139) ends it.
#   bash scripts/gpu_r4.sh TAG STEP...     steps: expm check ml mlab stamps probe ref
# Output: gpurun_out/TAG_<step>.log (+ json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread"
run() {   # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/${T}_${name}.log" | grep -v amdgpu.ids
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) exit $rc ;; esac
  return 0
}
for s in "$@"; do
  case $s in
    expm)   run expm 300 $PYT tests/test_gpu_parity.py -k "expm or manifold or wave or selection" ;;
    check)  run check 200 python -u scripts/wave_check.py --N 600 --epochs 1 --seed 1 ;;
    ml)     run ml 400 $PYT tests/test_gpu_movielens.py tests/test_gpu_quality.py -k "movielens" ;;
    mlab)   run mlold 200 env GPTSGLD_LIB=gpt_amd/libgptsgld_head.so python -u scripts/ml_ab.py
            run mlnew 200 python -u scripts/ml_ab.py
            run mlbench 300 python -u bench.py --workload movielens ;;
    chainab) run chainold 300 env GPTSGLD_LIB=gpt_amd/libgptsgld_head.so python -u bench.py --no-cpu-baseline --no-single-chain --steps 1000
            run chainnew 300 python -u bench.py --no-cpu-baseline --no-single-chain --steps 1000 ;;
    stamps) run stamps16 200 python -u scripts/wave_stamps.py --chains 16 --steps 4 --out gpurun_out/${T}_stamps16.json
            run stamps256 200 python -u scripts/wave_stamps.py --chains 256 --steps 4 --out gpurun_out/${T}_stamps256.json ;;
    probe)  run probe 300 python -u scripts/wave_probe.py --chains 256,10 --engines wave --steps 200 --out gpurun_out/${T}_probe.json ;;
    quality) run quality 900 $PYT tests/test_gpu_quality.py tests/test_gpu_fullsize.py -k "not movielens" ;;
    ref)    run ref 600 python -u bench.py --workload kin40k_ref ;;
    refprof) run refprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ref -o ref -- python -u bench.py --workload kin40k_ref --no-cpu-baseline --epochs 20 ;;
    mlprof) run mlprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ml -o ml -- python -u bench.py --workload movielens --no-cpu-baseline --epochs 40 ;;
    *) echo "unknown step $s" ;;
  esac
done
