"""Summarise a rocprofv3 --hip-trace rocpd database: the HIP API calls that block the host
(long durations) and the memcpy / synchronize calls, with their time relative to kernels.
    python tools/hip_trace_summary.py run_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print("tables/views:", [t for t in tables if not t.startswith("rocpd_info")][:40])
view = "regions" if "regions" in tables else None
if view is None:
    sys.exit(0)
cols = [r[1] for r in c.execute(f"pragma table_info({view})")]
print("regions cols:", cols)
rows = c.execute(f"select name, start, end, category from {view}").fetchall()
from collections import Counter, defaultdict
agg = defaultdict(lambda: [0, 0.0, 0.0])
for n, s, e, cat in rows:
    a = agg[n]
    a[0] += 1
    a[1] += (e - s) / 1e6
    a[2] = max(a[2], (e - s) / 1e6)
print("HIP API totals (calls, total ms, max ms):")
for n, (k, t, mx) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"  {n[:60]:60s} {k:7d} {t:10.2f} {mx:9.2f}")
print("calls longer than 1 ms (last 40):")
longs = [(s, e, n) for n, s, e, cat in rows if e - s > 1_000_000]
for s, e, n in sorted(longs)[-40:]:
    print(f"  {s / 1e6:14.3f} {(e - s) / 1e6:8.2f} ms  {n}")
