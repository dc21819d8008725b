"""Per-kernel time of one step of a rocprofv3 kernel trace (steps delimited by the patchify
kernel, which runs twice per step: teacher and student towers).
    python tools/step_breakdown.py run_results.db [top]"""
import collections
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sorted(c.execute("select name, start, end from kernels").fetchall(), key=lambda r: r[1])
pat = [r[1] for r in rows if "k_patchify" in r[0]]
a, b = pat[-4], pat[-2]
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
