"""PMC values of the chain step kernel from scripts/pmc_chain.sh passes, per chain-step of all
chains: the sum over every chain_kernel dispatch of a pass divided by the steps that pass's bench
process ran (the chain engine runs up to one epoch of steps per launch, so per-dispatch medians
mix launches of different lengths)."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
vals, disp = {}, {}
for d in sorted(glob.glob(os.path.join(out, "p*"))):
    if not os.path.isdir(d):
        continue
    steps = None
    try:
        last = [l for l in open(d + ".log") if l.startswith("{")][-1]
        steps = json.loads(last)["roofline"]["steps_run_per_chain"]
    except Exception:
        pass
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "chain_kernel" in row["Kernel_Name"]:
                    c = row["Counter_Name"]
                    vals[c] = vals.get(c, 0.0) + float(row["Counter_Value"])
                    disp[c] = (disp.get(c, (0, None))[0] + 1, steps)
for k in sorted(vals):
    n, steps = disp[k]
    if steps:
        print("%-24s %16.0f per step  (%d dispatches, %d steps)" % (k, vals[k] / steps, n, steps))
    else:
        print("%-24s %16.0f total  (%d dispatches, steps unknown)" % (k, vals[k], n))
