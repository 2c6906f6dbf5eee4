"""Kernel summary (rocprofv3 --kernel-trace --stats results database) as CSV for profiles/:

    python scripts/prof_summary.py gpurun_out/TAG_prof_ref/ref_results.db profiles/r4_ref_kernel_stats.csv

Columns: kernel name, calls, total / average / min / max duration (ns), share of kernel time.
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], "%.1f" % r[3], r[4], r[5], "%.3f" % (100.0 * r[2] / tot)])
    for r in rows[:6]:
        print("%-90s %6d calls  avg %10.1f us  %5.1f%%" % (r[0][:90], r[1], r[3] / 1e3, 100.0 * r[2] / tot))


if __name__ == "__main__":
    main()
