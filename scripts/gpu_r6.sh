#!/bin/bash
# One GPU session of round-6 checks, each step under its own time limit; a test failure (rc 1) is
# logged and the session goes on, a time limit / abort / segfault (124, 137, 134, 139) ends it.
#   bash scripts/gpu_r6.sh TAG STEP...
# Output: gpurun_out/TAG_<step>.log (+ profiles under gpurun_out/TAG_prof_*)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -q -x --timeout 200 --timeout-method thread"
run() {   # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/${T}_${name}.log" | grep -v amdgpu.ids | cut -c1-400
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) exit $rc ;; esac
  return 0
}
RP="rocprofv3 --kernel-trace --stats --output-format csv"
squeeze() {   # gzip the kernel traces of a profile directory (gpurun merges back at most 64 MiB)
  for f in "gpurun_out/${T}_prof_$1"/*kernel_trace.csv; do [ -f "$f" ] && gzip -f "$f"; done
  return 0
}
DF="python -u bench.py --gpus 1 --steps 20 --warmup 5"
for s in "$@"; do
  case $s in
    tests)    run tests 400 $PYT tests ;;
    driver)   for i in 1 2 3; do run driver$i 200 $DF; done ;;
    driver1)  run driver1 200 $DF ;;
    quick)    for i in 1 2 3; do run quick$i 200 $DF --no-cpu-baseline --no-single-chain; done ;;
    warmab)   for i in 1 2 3; do run wa1000_$i 200 $DF --no-cpu-baseline --no-single-chain --clock-warm-ms 1000; run wa2500_$i 200 $DF --no-cpu-baseline --no-single-chain --clock-warm-ms 2500; done ;;
    long)     run long 300 python -u bench.py --steps 2000 --warmup 200 --no-cpu-baseline ;;
    profdf)   run profdf 300 $RP -d gpurun_out/${T}_prof_df -o run -- $DF --no-cpu-baseline --no-single-chain; squeeze df ;;
    ref)      run ref 400 python -u bench.py --workload kin40k_ref --no-cpu-baseline ;;
    profref)  run profref 500 $RP -d gpurun_out/${T}_prof_ref -o run -- python -u bench.py --workload kin40k_ref --no-cpu-baseline --no-single-chain; squeeze ref ;;
    ml)       run ml 400 python -u bench.py --workload movielens ;;
    mltests)  run mltests 300 $PYT tests/test_gpu_movielens.py ;;
    mlstamps) run mlstamps 300 python -u scripts/ml_stamps.py ;;
    mlwstamps) run mlwstamps 300 env GPTSGLD_LIB=gpt_amd/libgptsgld_diag.so python -u scripts/ml_stamps.py ;;
    mlab)     for i in 1 2; do run mlab_head$i 300 python -u bench.py --workload movielens --no-cpu-baseline; run mlab_var$i 300 env GPTSGLD_LIB=gpt_amd/libgptsgld_var.so python -u bench.py --workload movielens --no-cpu-baseline; done ;;
    predab)   run predtests 300 $PYT tests/test_gpu_parity.py -k "pred" ; for i in 1 2; do run predab_head$i 200 python -u scripts/time_pred.py --S 224 --n 150 --r 20 --vphases rows; run predab_var$i 200 env GPTSGLD_LIB=gpt_amd/libgptsgld_var.so python -u scripts/time_pred.py --S 224 --n 150 --r 20 --vphases rows; done ;;
    mlnocpu)  run mlnocpu 300 python -u bench.py --workload movielens --no-cpu-baseline ;;
    pp)       run pp 400 python -u bench.py --workload powerplant --no-cpu-baseline ;;
    timeline) run timeline 300 env GPTSGLD_LIB=gpt_amd/libgptsgld_tl.so python -u scripts/timeline.py --out gpurun_out/${T}_timeline.json ;;
    host)     run host 300 python -u scripts/host_overhead.py --out gpurun_out/${T}_host.json ;;
    hostspin) run hostspin 300 python -u scripts/host_overhead.py --spin-flags --out gpurun_out/${T}_hostspin.json ;;
    hostaw)   run hostaw 300 env ROC_ACTIVE_WAIT_TIMEOUT=200 python -u scripts/host_overhead.py --out gpurun_out/${T}_hostaw.json ;;
    stamps)   run stamps 300 env GPTSGLD_LIB=gpt_amd/libgptsgld_diag.so python -u scripts/phase_stamps.py --engine chain --chains 256 --steps 30 ;;
    round)    run round 900 env TAG=${T} bash scripts/profile_round.sh --steps 20 --warmup 5 ;;
    pmc)      run pmc 900 env TAG=${T} bash scripts/pmc_chain.sh ;;
    single)   run single 300 python -u scripts/single_chain_ab.py ;;
    smoke)    run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    *)        echo "unknown step $s"; exit 2 ;;
  esac
done
