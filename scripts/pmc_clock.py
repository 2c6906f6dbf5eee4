"""Effective clock and MFMA busy fraction per dispatch from a rocprofv3 --pmc pass of
GRBM_GUI_ACTIVE and SQ_VALU_MFMA_BUSY_CYCLES (with --kernel-trace for the durations).

    python scripts/pmc_clock.py DIR/<name>_counter_collection.csv [--match mfma,vphase] [--simds 1024]

Effective clock = GRBM_GUI_ACTIVE / 8 (the counter is summed over the 8 XCDs) / kernel wall time
(MI355X_MICROARCH.md, "DVFS give-back"); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x clock
cycles of the dispatch).
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("counters")
    ap.add_argument("--match", default="mfma,vphase")
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args()
    pats = a.match.split(",")
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(a.counters)):
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        d = agg.setdefault(key, {"start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print("%-10s %-48s %10s %9s %10s" % ("dispatch", "kernel", "ms", "clock GHz", "mfma busy"))
    for (disp, name), d in agg.items():
        if not any(p in name for p in pats):
            continue
        dur = (d["end"] - d["start"]) * 1e-9
        clk = d.get("GRBM_GUI_ACTIVE", 0.0) / 8 / dur
        busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (a.simds * clk * dur) if clk > 0 else 0.0
        short = name.split("(")[0].replace("void ", "")[:48]
        print("%-10s %-48s %10.3f %9.3f %10.3f" % (disp, short, dur * 1e3, clk / 1e9, busy))


if __name__ == "__main__":
    main()
