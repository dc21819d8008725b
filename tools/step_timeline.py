"""Coarse timeline of one concurrent training step from a rocprofv3 kernel trace (the window
between the last two AdamW launches): per time bucket, which streams run what, and a CU-fill
estimate (sum over running kernels of min(1, workgroups / 256), capped at 1 — a big GEMM
grid counts as full, a 115-tile GEMM as 0.45).
    python tools/step_timeline.py run_results.db [bucket_ms]"""
import collections
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
bucket = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
rows = c.execute("select name, start, end, stream_id, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z "
                 "from kernels").fetchall()
rows.sort(key=lambda r: r[1])
opt = [r[1] for r in rows if "k_adamw" in r[0]]
a, b = opt[-2], opt[-1]
rr = [r for r in rows if a <= r[1] < b]


def short(n):
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)", "")).replace("void ", "").replace("kd::::", "")
    n = n.replace("at::native::", "")
    return n[:28]


streams = sorted({r[3] for r in rr})
nb = int((b - a) / 1e6 / bucket) + 1
fill = [0.0] * nb
busy = {s: [0.0] * nb for s in streams}
names = {s: [collections.Counter() for _ in range(nb)] for s in streams}
for n, s, e, st, gx, gy, gz, wx, wy, wz in rr:
    wgs = max(1, (gx * gy * gz) // max(1, wx * wy * wz))
    f = min(1.0, wgs / 256)
    t0, t1 = (s - a) / 1e6, (min(e, b) - a) / 1e6
    k = int(t0 / bucket)
    while k < nb and k * bucket < t1:
        lo, hi = max(t0, k * bucket), min(t1, (k + 1) * bucket)
        if hi > lo:
            fill[k] += f * (hi - lo) / bucket
            busy[st][k] += (hi - lo) / bucket
            names[st][k][short(n)] += hi - lo
        k += 1
print(f"step {(b - a) / 1e6:.2f} ms; streams {streams}; mean CU fill {sum(min(1, x) for x in fill) / nb:.3f}")
for k in range(nb):
    cols = []
    for s in streams:
        if busy[s][k] > 0.02:
            top = names[s][k].most_common(1)[0][0]
            cols.append(f"s{s}:{busy[s][k]:.2f} {top}")
    print(f"{k * bucket:7.1f} fill {min(1.0, fill[k]):.2f} | " + " | ".join(cols))
