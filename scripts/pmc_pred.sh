#!/bin/bash
# MFMA busy cycles and GPU-active cycles of the stacked-sample prediction GEMM (one --pmc pass,
# kernel-trace only), for the MFMA-utilisation figure in DESIGN.md §3.3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_pred -o run -- python3 scripts/time_pred.py --tiles 44 --reps 1 > gpurun_out/pmc_pred.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_pred.log; exit $rc; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/pmc_pred/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "pred_temp_mfma" in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
tr = {r["Dispatch_Id"]: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open("gpurun_out/pmc_pred/run_kernel_trace.csv"))}
for d, c in agg.items():
    ns = tr.get(d, 0)
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    print("dispatch %s: %.3f ms, MFMA busy %.4g, GUI active/8 %.4g cyc, clock %.2f GHz, MFMA busy per SIMD-cycle %.3f"
          % (d, ns / 1e6, c["SQ_VALU_MFMA_BUSY_CYCLES"], cyc, cyc / max(ns, 1), c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc)))
PY
