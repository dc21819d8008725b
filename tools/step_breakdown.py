"""Per-kernel time of one training step of a rocprofv3 kernel trace: the window between the
last two AdamW launches (one per optimizer step; the teacher-forward rate pass bench.py
runs after the timed steps has no AdamW).
    python tools/step_breakdown.py run_results.db [top]"""
import collections
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sorted(c.execute("select name, start, end from kernels").fetchall(), key=lambda r: r[1])
opt = [r[1] for r in rows if "k_adamw" in r[0]]
a, b = opt[-2], opt[-1]
rr = [r for r in rows if a <= r[1] < b]
agg = collections.defaultdict(lambda: [0, 0])
for n, s, e in rr:
    k = re.sub(r"\(.*", "", n.replace("(anonymous namespace)", "")).replace("void ", "").replace("kd::::", "")
    agg[k][0] += e - s
    agg[k][1] += 1
tot = sum(v[0] for v in agg.values())
print(f"step span {(b - a) / 1e6:.2f} ms, kernel sum {tot / 1e6:.2f} ms")
for k, (t, n) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
    print(f"{t / 1e6:8.2f} ms {100 * t / tot:5.1f}% {n:5d}  {k[:90]}")
