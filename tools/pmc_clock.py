"""Effective shader clock per kernel family from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass with
--kernel-trace (MI355X_MICROARCH.md 'DVFS give-back': clock ~ GRBM_GUI_ACTIVE / 8 / kernel wall
time; rocprofv3 sums the counter over the 8 XCDs; reads high on dispatches < 0.3 ms).
    python tools/pmc_clock.py <rocprofv3 output dir>"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])   # launches, sum cycles/8, sum ns
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        if ns <= 0:
            continue
        n = r["Kernel_Name"].replace("kd::(anonymous namespace)::", "").split("(")[0][:60]
        a = agg[n]
        a[0] += 1
        a[1] += float(r["Counter_Value"]) / 8.0
        a[2] += ns
tot_c = sum(a[1] for a in agg.values())
tot_t = sum(a[2] for a in agg.values())
print(f"all kernels: {tot_t / 1e6:.1f} ms, effective clock {tot_c / tot_t:.3f} GHz")
for n, (k, c, t) in sorted(agg.items(), key=lambda kv: -kv[1][2])[:25]:
    print(f"{t / 1e6:9.2f} ms {k:5d}  {c / t:6.3f} GHz  {n}")
