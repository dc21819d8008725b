"""Summarise tools/pmc_vs_blas.sh: per program and kernel, the average wall time, TF/s,
effective clock (GRBM_GUI_ACTIVE / 8 / wall: rocprofv3 sums the counter over the 8 XCDs),
MFMA-busy cycles per FLOP and per wall cycle, and SQ busy / wave cycles.
    python tools/pmc_vs_blas.py gpurun_out/pmc_blas"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*_*x*x*"))):
    if not os.path.isdir(d):
        continue
    prog, shape = os.path.basename(d).split("_", 1)
    M, N, K = (int(x) for x in shape.split("x"))
    flop = 2.0 * M * N * K
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0][-60:]
            ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            agg[(name, r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
            agg[(name, r["Dispatch_Id"])]["ns"] = [ns]
    per = collections.defaultdict(list)
    for (name, _), c in agg.items():
        if "GRBM_GUI_ACTIVE" not in c or c["ns"][0] < 100e3:   # the GEMM dispatches only (>= 0.1 ms)
            continue
        per[name].append({k: sum(v) for k, v in c.items()})
    for name, rows in per.items():
        n = len(rows)
        ns = sum(r["ns"] for r in rows) / n
        grbm = sum(r["GRBM_GUI_ACTIVE"] for r in rows) / n
        mfma = sum(r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for r in rows) / n
        wave = sum(r.get("SQ_WAVE_CYCLES", 0) for r in rows) / n
        busy = sum(r.get("SQ_BUSY_CYCLES", 0) for r in rows) / n
        clk = grbm / 8 / ns
        fetch = sum(r.get("FETCH_SIZE", 0) for r in rows) / n * 2048.0   # KB, x2 (gfx950 wide-read correction)
        write = sum(r.get("WRITE_SIZE", 0) for r in rows) / n * 1024.0
        print(f"{prog:5s} {shape:18s} {name[-44:]:44s} n={n:2d} {ns / 1e3:8.1f} us {flop / ns / 1e3:7.1f} TF/s "
              f"clock {clk:5.3f} GHz  FLOP/cycle {flop / (grbm / 8):9.0f}  MFMA-busy/FLOP {mfma / flop * 1e3:7.4f}e-3  "
              f"MFMA-busy/wall-cycle {mfma / (grbm / 8):8.1f}  SQ_BUSY/wall-cycle {busy / (grbm / 8):6.2f}  "
              f"wave-cycles/FLOP {wave / flop * 1e3:7.4f}e-3  FETCH {fetch / 1e9:6.3f} GB  WRITE {write / 1e9:6.3f} GB "
              f"(A + B once: {(M + N) * K * 2 / 1e9:6.3f} GB)")
