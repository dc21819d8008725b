"""Summarise a rocprofv3 rocpd database (kernel-trace) into a per-kernel stats CSV.
    python tools/prof_stats.py run_results.db [out.csv]"""
import csv
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else "kernel_name"
rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
agg = {}
for n, s, e in rows:
    d = (e - s) / 1e3
    a = agg.setdefault(n, [0, 0.0, 1e30, 0.0])
    a[0] += 1; a[1] += d; a[2] = min(a[2], d); a[3] = max(a[3], d)
tot = sum(a[1] for a in agg.values())
out = sorted(agg.items(), key=lambda kv: -kv[1][1])
w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "MinUs", "MaxUs", "Percentage"])
for n, (k, t, mn, mx) in out:
    w.writerow([n, k, f"{t:.1f}", f"{t / k:.2f}", f"{mn:.2f}", f"{mx:.2f}", f"{100 * t / tot:.2f}"])
