"""Summarise rocprofv3 --pmc CSVs: python tools/pmc_summary.py DIR [DIR ...] (kernel-name filter: gemm|Cijk)"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/p*/p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "gemm" not in n and "Cijk" not in n:
                continue
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    print(d)
    for k, v in sorted(m.items()):
        print(f"  {k:28s} {v:.4g}")
    if "SQ_WAVE_CYCLES" in m:
        w = m["SQ_WAVE_CYCLES"]
        print(f"  -> wait_any {m['SQ_WAIT_ANY'] / w:.2f} wait_inst {m['SQ_WAIT_INST_ANY'] / w:.2f} active {m['SQ_ACTIVE_INST_ANY'] / w:.2f}"
              f"  mfma_busy/(gui/8*1024) {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f}")
