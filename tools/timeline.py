"""GPU timeline of a rocprofv3 kernel trace: busy (union of kernel intervals) vs idle time
over the last N steps' window, and the kernels that run alone longest.
    python tools/timeline.py run_results.db [t_first_frac]"""
import sqlite3
import sys

db = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else "kernel_name"
rows = sorted(c.execute(f"select {name_col}, start, end from kernels").fetchall(), key=lambda r: r[1])
t0, t1 = rows[0][1], max(r[2] for r in rows)
lo = t0 + (t1 - t0) * frac
rows = [r for r in rows if r[1] >= lo]
busy, cur_s, cur_e = 0, None, None
for _, s, e in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = max(r[2] for r in rows) - rows[0][1]
ksum = sum(e - s for _, s, e in rows)
print(f"window {span / 1e6:.1f} ms: GPU busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f}%), "
      f"sum of kernel time {ksum / 1e6:.1f} ms (concurrency {ksum / max(busy, 1):.2f}x), {len(rows)} kernels")
