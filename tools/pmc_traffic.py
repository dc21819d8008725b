"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_bench.sh) into per-kernel HBM bytes.

    python tools/pmc_traffic.py gpurun_out/pmc_bench > traffic.json

Corrections (MI355X_MICROARCH.md, HBM section): rocprofv3 reports both counters in KB; on
gfx950 FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) streaming read,
global_load and buffer_load ... lds alike, so it is doubled; WRITE_SIZE is exact for 16-B
stores. Averages are over every launch of a kernel (warm-up and measured steps alike: the
per-launch traffic of one GEMM shape does not depend on the step).
"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]


def load(pass_dir, counter):
    per = collections.defaultdict(list)
    for f in glob.glob(f"{root}/{pass_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return per


def short(n):
    return n.replace("kd::(anonymous namespace)::", "").split("(")[0][:100]


def is_roofline_kernel(n):   # bench.py's roofline kernel: the fused gate|up + SwiGLU GEMM (v8 GLU build)
    return "k_gemm8<false, false, 4>" in n


fetch, write = load("p1", "FETCH_SIZE"), load("p2", "WRITE_SIZE")
out = {"note": "bytes per launch; FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE as reported",
       "kernels": {}}
fw_f, fw_w = [], []
for n in sorted(set(fetch) | set(write)):
    f, w = fetch.get(n, []), write.get(n, [])
    k = short(n)
    e = out["kernels"].setdefault(k, dict(launches=0, fetch_bytes=0.0, write_bytes=0.0))
    e["launches"] = max(len(f), len(w))
    e["fetch_bytes"] = 2.0 * sum(f) / max(len(f), 1)
    e["write_bytes"] = sum(w) / max(len(w), 1)
    if is_roofline_kernel(n):
        fw_f += f
        fw_w += w
if fw_f:
    fb = 2.0 * sum(fw_f) / len(fw_f)
    wb = sum(fw_w) / max(len(fw_w), 1)
    out["roofline_kernel"] = dict(launches=len(fw_f), fetch_bytes=fb, write_bytes=wb, traffic_bytes=fb + wb)
json.dump(out, sys.stdout, indent=1)
