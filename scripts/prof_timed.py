"""The timed region of a bench.py run, isolated from its rocprofv3 kernel trace.

bench.py launches one marker dispatch (torch.cuda._sleep: a spin kernel) right before its timed
region and one right after it, both outside the timed wall clock.  Every dispatch that starts
after the first marker ends and ends before the second begins is a timed step's kernel.  Per step
of all chains this reports (a) the device span (first timed start to last timed end, what the
bench's hipEvent pair measures) and (b) the kernels' summed durations, per kernel name.

    python scripts/prof_timed.py TRACE.csv --steps 20 [--bench LINE.json] [--out OUT.json]
"""
import argparse
import gzip
import csv
import json
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True, help="timed steps of the bench run")
    ap.add_argument("--marker", default="spin", help="substring of the marker kernel's name")
    ap.add_argument("--bench", default=None, help="the bench's JSON line, to compare against")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    opener = gzip.open if args.trace.endswith(".gz") else open
    rows = list(csv.DictReader(opener(args.trace, "rt")))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    marks = [r for r in rows if args.marker in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit("fewer than two marker dispatches (%r) in the trace" % args.marker)
    lo, hi = marks[0]["e"], marks[1]["s"]
    timed = [r for r in rows if r["s"] > lo and r["e"] < hi and args.marker not in r["Kernel_Name"]]
    if not timed:
        sys.exit("no dispatch between the markers")
    span_ns = max(r["e"] for r in timed) - min(r["s"] for r in timed)
    per = {}
    for r in timed:
        k = r["Kernel_Name"].split("(")[0]
        d = per.setdefault(k, dict(calls=0, total_ns=0, grid_x=int(r["Grid_Size_X"]),
                                   workgroup_x=int(r["Workgroup_Size_X"])))
        d["calls"] += 1
        d["total_ns"] += r["e"] - r["s"]
    busy_ns = sum(d["total_ns"] for d in per.values())
    out = dict(trace=args.trace, steps=args.steps, dispatches=len(timed),
               span_us_per_step=span_ns / 1e3 / args.steps,
               kernel_us_per_step=busy_ns / 1e3 / args.steps,
               kernels={k: dict(d, us_per_step=d["total_ns"] / 1e3 / args.steps,
                                avg_us=d["total_ns"] / 1e3 / d["calls"]) for k, d in per.items()})
    if args.bench:
        line = json.loads(open(args.bench).read().strip().splitlines()[-1])
        ku = line["roofline"]["kernel_us"]
        out["bench"] = dict(kernel_us=ku, ms_per_step=line["ms_per_step"],
                            frac=line["roofline"]["frac"],
                            span_vs_bench_kernel_us=out["span_us_per_step"] / ku - 1.0,
                            frac_from_profile_span=line["roofline"]["frac"] * ku
                            / out["span_us_per_step"])
    print(json.dumps(out, indent=1))
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
