"""Median per-dispatch PMC values of the chain step kernel from scripts/pmc_chain.sh passes."""
import csv
import glob
import os
import statistics
import sys

out = sys.argv[1]
vals = {}
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if "chain_kernel" in row["Kernel_Name"]:
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
for k in sorted(vals):
    print("%-24s %16.0f  (%d dispatches)" % (k, statistics.median(vals[k]), len(vals[k])))
