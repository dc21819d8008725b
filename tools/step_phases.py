"""Phases of one KD step in a rocprofv3 kernel trace (concurrent bench): per stream the busy
time, and the wall time of the phases delimited by marker kernels.
    python tools/step_phases.py run_results.db
Markers: the first k_patchify of a step (forward start), k_row_stats (loss start),
k_loss_grad end (backward start), the last kernel before the next step's first patchify."""
import collections
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = sorted(c.execute("select name, start, end, stream_id from kernels").fetchall(), key=lambda r: r[1])
pat = [r[1] for r in rows if "k_patchify" in r[0]]
starts = pat[::2]
a, b = starts[-3], starts[-2]   # the second-to-last complete step
rr = [r for r in rows if a <= r[1] < b]
span = b - a
print(f"step {span / 1e6:.2f} ms, {len(rr)} kernels")


def short(n):
    return re.sub(r"\(.*", "", n.replace("(anonymous namespace)", "")).replace("void ", "").replace("kd::::", "")[:50]


per_stream = collections.defaultdict(lambda: [0, 0, None, None])
for n, s, e, sid in rr:
    ps = per_stream[sid]
    ps[0] += e - s
    ps[1] += 1
    ps[2] = s if ps[2] is None else min(ps[2], s)
    ps[3] = e if ps[3] is None else max(ps[3], e)
for sid, (t, n, s0, e0) in sorted(per_stream.items()):
    first = next(short(r[0]) for r in rr if r[3] == sid)
    print(f"  stream {sid}: {n:5d} kernels, busy {t / 1e6:7.2f} ms, active {(s0 - a) / 1e6:7.2f} .. {(e0 - a) / 1e6:7.2f} ms"
          f"  (first: {first})")
rs = next(r for r in rr if "k_row_stats" in r[0])
lg = next(r for r in rr if "k_loss_grad" in r[0])
print(f"  forward (teacher + student): 0 .. {(rs[1] - a) / 1e6:.2f} ms")
print(f"  loss: {(rs[1] - a) / 1e6:.2f} .. {(lg[2] - a) / 1e6:.2f} ms")
print(f"  backward + optimizer: {(lg[2] - a) / 1e6:.2f} .. {span / 1e6:.2f} ms")
# the main stream's idle gaps > 50 us (waiting on other streams or the host)
main_sid = rs[3]
ms = [r for r in rr if r[3] == main_sid]
gaps = [(ms[i + 1][1] - ms[i][2], short(ms[i][0]), short(ms[i + 1][0]), (ms[i][2] - a) / 1e6)
        for i in range(len(ms) - 1) if ms[i + 1][1] - ms[i][2] > 50_000]
print(f"  main stream {main_sid}: {len(gaps)} gaps > 50 us, total {sum(g[0] for g in gaps) / 1e6:.2f} ms")
for g in sorted(gaps, reverse=True)[:12]:
    print(f"    {g[0] / 1e3:8.1f} us at {g[3]:7.2f} ms after {g[1]} -> {g[2]}")
