#!/bin/bash
# One GPU session of round-5 checks, each step under its own time limit; a test failure (rc 1) is
# logged and the session goes on, a time limit / abort / segfault (124, 137, 134, 139) ends it.
#   bash scripts/gpu_r5.sh TAG STEP...
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
  tail -4 "gpurun_out/${T}_${name}.log" | grep -v amdgpu.ids
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) exit $rc ;; esac
  return 0
}
RP="rocprofv3 --kernel-trace --stats --output-format csv"
squeeze() {   # gzip the kernel traces of a profile directory (gpurun merges back at most 64 MiB)
  for f in "gpurun_out/${T}_prof_$1"/*kernel_trace.csv; do [ -f "$f" ] && gzip -f "$f"; done
  return 0
}
for s in "$@"; do
  case $s in
    tests)   run tests 400 $PYT tests ;;
    newtests) run newtests 300 $PYT tests/test_gpu_parity.py tests/test_gpu_movielens.py -k "environment or selection or movielens or cf" ;;
    repro0)  run repro0 300 env GPTSGLD_MAX_INFLIGHT=0 $RP -d gpurun_out/${T}_prof_repro0 -o repro -- python -u scripts/refprof_repro.py --maps gpurun_out/${T}_repro0_maps.txt ;;
    repro8)  run repro8 300 $RP -d gpurun_out/${T}_prof_repro8 -o repro -- python -u scripts/refprof_repro.py --maps gpurun_out/${T}_repro8_maps.txt ;;
    bench)   run bench 300 python -u bench.py ;;
    prof)    run prof 600 $RP -d gpurun_out/${T}_prof_bench -o bench -- python -u bench.py --no-cpu-baseline; squeeze bench ;;
    sweep500) run sweep500 600 python -u scripts/kin40k_step_sweep.py --n 500 --r 5 --epsw 5e-6,1e-5,1.2e-5,1e-4 --epsU 1e-8,3e-8,1e-7,3e-7 --out gpurun_out/${T}_sweep500.json ;;
    sweep150) run sweep150 600 python -u scripts/kin40k_step_sweep.py --n 150 --r 5 --epsw 5e-6,1e-5,3e-5,1e-4 --epsU 1e-8,3e-8,1e-7,3e-7 --out gpurun_out/${T}_sweep150.json ;;
    sweep150r20) run sweep150r20 600 python -u scripts/kin40k_step_sweep.py --n 150 --r 20 --epsw 1e-5,3e-5,1e-4,2e-4 --epsU 1e-8,3e-8,1e-7,3e-7 --out gpurun_out/${T}_sweep150r20.json ;;
    ref)     run ref 600 python -u bench.py --workload kin40k_ref ;;
    refprof) run refprof 600 $RP -d gpurun_out/${T}_prof_ref -o ref -- python -u bench.py --workload kin40k_ref --no-cpu-baseline; squeeze ref ;;
    ml)      run ml 300 python -u bench.py --workload movielens ;;
    mlprof)  run mlprof 600 $RP -d gpurun_out/${T}_prof_ml -o ml -- python -u bench.py --workload movielens --no-cpu-baseline; squeeze ml ;;
    pp)      run pp 300 python -u bench.py --workload powerplant ;;
    quality) run quality 900 $PYT tests/test_gpu_quality.py tests/test_gpu_fullsize.py ;;
    gibbsprof) run gibbsprof 300 $RP -d gpurun_out/${T}_prof_gibbs -o gibbs -- python -u scripts/time_gibbs.py --sweeps 40; squeeze gibbs ;;
    ppprof) run ppprof 600 $RP -d gpurun_out/${T}_prof_pp -o pp -- python -u bench.py --workload powerplant --no-cpu-baseline; squeeze pp ;;
    predclk) run predclk 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/${T}_prof_predclk -o predclk -- python -u scripts/time_pred.py --S 256 --tiles 44 --vphases pairs ;;
    pair) run pair 300 python -u bench.py --epsw 1e-4 --epsU 1e-8 --no-cpu-baseline --no-single-chain ;;
    hq) run hq 300 $PYT tests/test_gpu_quality.py -k "bench_shape or powerplant_config2_converged" ;;
    mltests) run mltests 400 $PYT tests/test_gpu_movielens.py tests/test_gpu_tgp.py tests/test_gpu_quality.py -k "movielens or tgp or gibbs or bench_shape" ;;
    gibbs) run gibbs 300 python -u scripts/time_gibbs.py --sweeps 200 ;;
    pred20) run pred20 300 python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows ;;
    pred5) run pred5 300 python -u scripts/time_pred.py --S 256 --tiles 44 --vphases pairs,rows ;;
    predtests) run predtests 300 $PYT tests/test_gpu_parity.py -k "pred" ;;
    wavetests) run wavetests 400 $PYT tests/test_gpu_parity.py -k "expm or wave or manifold or selection or injected or nan or multichain or epoch_order" ;;
    expm) run expm 200 python -u scripts/expm_bench.py --nn 40 ;;
    wstamps) run wstamps 200 python -u scripts/wave_stamps.py --chains 256 --steps 4 --out gpurun_out/${T}_wstamps.json ;;
    refq) run refq 300 python -u bench.py --workload kin40k_ref --no-cpu-baseline --epochs 20 ;;
    mlstamps) run mlstamps 300 python -u scripts/ml_stamps.py ;;
    mlstamps0) run mlstamps0 300 env GPTSGLD_CF_LAZY=0 python -u scripts/ml_stamps.py ;;
    mlab) for v in 0 1 0 1; do run mlab_$v 300 env GPTSGLD_CF_LAZY=$v python -u bench.py --workload movielens --no-cpu-baseline; done ;;
    wvab) for v in product u2 u4 product; do
            if [ $v = product ]; then L=gpt_amd/libgptsgld.so; else L=gpt_amd/libgptsgld_abl_$v.so; fi
            run wvab_$v 200 env GPTSGLD_LIB=$L python -u scripts/wave_probe.py --chains 256 --engines wave --steps 400
          done ;;
    chainab) for v in head new head new; do
            if [ $v = head ]; then L=gpt_amd/libgptsgld_head.so; else L=gpt_amd/libgptsgld.so; fi
            run chainab_$v 300 env GPTSGLD_LIB=$L python -u bench.py --no-cpu-baseline --no-single-chain --steps 1000
          done ;;
    chaintests) run chaintests 400 $PYT tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "chain or kin40k or powerplant or multichain or injected or nan or epoch_order or grad or trajectory" ;;
    predab) for v in head new head new; do
              if [ $v = head ]; then L=gpt_amd/libgptsgld_head.so; else L=gpt_amd/libgptsgld.so; fi
              run predab5_$v 200 env GPTSGLD_LIB=$L python -u scripts/time_pred.py --S 256 --tiles 44 --vphases pairs --reps 5
              run predab20_$v 200 env GPTSGLD_LIB=$L python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows --reps 5
            done ;;
    pred20prof) run pred20prof 200 $RP -d gpurun_out/${T}_prof_pred20 -o p20 -- python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows --reps 3 ;;
    pred20pmc) run pred20pmc 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/${T}_prof_p20pmc -o p20pmc -- python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows --reps 1 &&
               run pred20pmc2 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${T}_prof_p20pmc2 -o p20pmc2 -- python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows --reps 1 ;;
    scstamps) run scstamps 200 python -u scripts/phase_stamps.py --chains 1 --steps 30 ;;
    gridsync) run gridsync 120 ./diagbin/gridsync_bench ;;
    rowsabl) for a in 0 1 2 0; do run rowsabl_$a 200 env GPTSGLD_ROWS_ABL=$a $RP -d gpurun_out/${T}_prof_rabl$a -o r -- python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows --reps 3; done ;;
    allocab) for a in pool plain pool plain; do run allocab_$a 200 env GPTSGLD_PRED_ALLOC=$a $RP -d gpurun_out/${T}_prof_alloc_$a -o r -- python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows --reps 3; done ;;
    nwab) for a in 8 16 8 16; do run nwab_$a 200 env GPTSGLD_PRED_ROWS_NW=$a $RP -d gpurun_out/${T}_prof_nw$a -o r -- python -u scripts/time_pred.py --S 224 --n 150 --r 20 --tiles 44 --vphases rows --reps 3; done ;;
    wvhead) for v in head new head new; do
              if [ $v = head ]; then L=gpt_amd/libgptsgld_head.so; else L=gpt_amd/libgptsgld.so; fi
              run wvhead_$v 200 env GPTSGLD_LIB=$L python -u scripts/wave_probe.py --chains 256 --engines wave --steps 400
            done ;;
    bailtest) run bailtest 300 $PYT tests/test_gpu_quality.py -k "bailouts_match" ;;
    chainsab) for c in 256 288 320; do run chainsab_$c 300 python -u bench.py --workload kin40k_ref --chains $c --no-cpu-baseline --no-single-chain; done ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $s" ;;
  esac
done
