"""Summarise a profile_round.sh run: kernel-trace stats and per-launch HBM traffic of the
dominant step kernel, written into profiles/.

    python scripts/pmc_summary.py gpurun_out/prof_r1b --tag r1b --key C256_n500_D8_r5_Q200_m50

Traffic per launch = (2·FETCH_SIZE + WRITE_SIZE) KiB: on gfx950 FETCH_SIZE counts half the bytes
of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM), which is how the step kernels read
the minibatch rows (global_load_lds_dwordx4); WRITE_SIZE is exact for 16-B stores and is used as
reported for the 8-B state stores (uncalibrated, small).
"""
import argparse
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, counter, match, grid=None):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and match in row["Kernel_Name"]:
                if grid is None or int(row["Grid_Size"]) == grid:
                    vals.append(float(row["Counter_Value"]))
    return vals


def timed_launches(path, match):
    """(grid size, durations in us) of the bench's timed launches: the largest grid of the
    kernel (bench.py also runs a one-chain latency pass of the same kernel)."""
    by = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if match in row["Kernel_Name"]:
                g = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
                by.setdefault(g, []).append(
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0)
    g = max(by)
    return g, by[g]


def steps_run(log):
    """Chain-steps per chain the profiled bench process ran (its JSON line), or None."""
    try:
        last = [l for l in open(log) if l.startswith("{")][-1]
        return json.loads(last)["roofline"].get("steps_run_per_chain")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--key", required=True, help="pmc_traffic.json key (bench config)")
    ap.add_argument("--kernel", default="chain_kernel", help="substring of the dominant kernel")
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    stats = os.path.join(args.outdir, "stats", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, "%s_kernel_stats.csv" % args.tag))
    avg_ns = None
    with open(stats) as f:
        for row in csv.DictReader(f):
            if args.kernel in row["Name"]:
                avg_ns = float(row["AverageNs"])
                name = row["Name"]
                calls = int(row["Calls"])
                break
    if avg_ns is None:
        sys.exit("kernel %s not in %s" % (args.kernel, stats))
    grid, durs = timed_launches(os.path.join(args.outdir, "stats", "run_kernel_trace.csv"),
                                args.kernel)
    fetch = per_dispatch(os.path.join(args.outdir, "fetch", "run_counter_collection.csv"),
                         "FETCH_SIZE", args.kernel, grid)
    write = per_dispatch(os.path.join(args.outdir, "write", "run_counter_collection.csv"),
                         "WRITE_SIZE", args.kernel, grid)
    fm, wm = statistics.median(fetch), statistics.median(write)
    # the chain engine runs up to one epoch of steps per launch: per-step figures are the sums
    # over every launch of the kernel divided by the steps the process ran
    ns = steps_run(os.path.join(args.outdir, "stats.log"))
    nf = steps_run(os.path.join(args.outdir, "fetch.log"))
    nw = steps_run(os.path.join(args.outdir, "write.log"))
    per_step = {}
    if ns and nf and nw:
        per_step = {
            "steps_run": ns,
            "avg_duration_us_per_step": sum(durs) / ns,
            "hbm_bytes_per_step": (2 * sum(fetch) / nf + sum(write) / nw) * 1024.0,
        }
    entry = {
        "kernel": name.split("(")[0].replace("void ", ""),
        "avg_duration_us_all_launches": avg_ns / 1000.0,
        "calls": calls,
        "timed_grid_threads": grid,
        "avg_duration_us": statistics.mean(durs),
        "timed_launches": len(durs),
        "FETCH_SIZE_KB_median": fm,
        "WRITE_SIZE_KB_median": wm,
        "launches": len(fetch),
        "correction": "gfx950 FETCH_SIZE counts half the bytes of 16-B/lane streaming reads "
                      "(MI355X_MICROARCH.md HBM): bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024",
        "hbm_bytes_per_launch": per_step.get("hbm_bytes_per_step", (2 * fm + wm) * 1024.0),
        "per_step": per_step,
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE --kernel-trace, separate passes "
                  "(scripts/profile_round.sh), tag %s" % args.tag,
    }
    pj = os.path.join(prof, "pmc_traffic.json")
    data = json.load(open(pj)) if os.path.exists(pj) else {}
    data[args.key] = entry
    json.dump(data, open(pj, "w"), indent=1)
    bj = os.path.join(args.outdir, "bench.json")
    if os.path.exists(bj):
        shutil.copy(bj, os.path.join(prof, "%s_bench.json" % args.tag))
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
