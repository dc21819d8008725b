"""Per kernel family of the serialized c1 step: time, MFMA utilisation, clock and HBM traffic, from
the rocprofv3 --pmc passes of tools/pmc_bench.sh mfma (north_star: "rocprof HBM GB/s and MFMA
utilisation against gfx950 peak").

    python tools/pmc_step.py gpurun_out/r05/pmc_bench > pmc_step.json

Passes (separate runs of the same serialized bench, bench.py --steps 2 --warmup 1 --serial):
  p1 FETCH_SIZE, p2 WRITE_SIZE (KB; FETCH_SIZE x2: the gfx950 wide-read correction, MI355X_MICROARCH.md)
  p3 GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES
Per dispatch: wall = End - Start (ns); cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs);
clock = cycles / wall.  SQ_VALU_MFMA_BUSY_CYCLES counts MFMA pipe cycles summed over the SIMDs
(32 per 32x32x16 bf16 MFMA, 16 per 16x16x32), so the matrix pipes' utilisation is
  mfma_util = MFMA_BUSY / (1024 SIMDs x cycles)            (256 CUs x 4 SIMDs)
and at the clock the chip held it corresponds to mfma_util x clock / 2.4 GHz of the 2.5 PF dense bf16
peak (the peak is quoted at 2.4 GHz).  A family's figures are sums over its dispatches (ratios of
sums), per step = / the 3 steps each pass runs.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import re
import sys

N_SIMD = 1024
PEAK_CLK = 2.4
STEPS = 3


def family(n: str) -> str:
    if "k_gemm8f8" in n:
        return "gemm fp8"
    m = re.search(r"k_gemm(8|3)<(?:\d+, \d+, )?(true|false), (true|false)(?:, (\d+))?", n)
    if m:
        amn, bmn, exp = m.group(2) == "true", m.group(3) == "true", int(m.group(4) or 0)
        if exp & 4:
            return "gemm fwd gate|up + SwiGLU (roofline kernel)"
        if exp & 32:
            return "gemm fwd lm_head + row stats"
        lay = {(False, False): "fwd (K x K)", (False, True): "dgrad (K x MN)", (True, True): "wgrad (MN x MN)",
               (True, False): "wgrad (MN x K)"}[(amn, bmn)]
        return f"gemm {lay}"
    if "k_gemm<" in n:
        return "gemm small (v1)"
    if "k_splitk_reduce" in n:
        return "gemm split-K reduce"
    if "k_attn_fwd" in n:
        return "attention fwd"
    if "k_attn" in n:
        return "attention bwd"
    if any(k in n for k in ("k_row_stats", "k_loss_grad", "k_ovr_mask", "k_count_valid", "k_finalize")):
        return "KD loss"
    if "k_norm" in n or "k_reduce_parts" in n:
        return "norms"
    if "k_adamw" in n:
        return "AdamW"
    if "k_qkv" in n or "k_swiglu" in n or "k_act_bwd" in n:
        return "qkv / activation (unfused)"
    if "k_colsum" in n:
        return "bias colsum"
    return "other"


def load(root, pas):
    """{dispatch id: {"name", "ns", counters...}} of one pass."""
    out = {}
    for f in glob.glob(f"{root}/{pas}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = out.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"],
                                                   "ns": float(r["End_Timestamp"]) - float(r["Start_Timestamp"])})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    root = sys.argv[1]
    p1, p2, p3 = load(root, "p1"), load(root, "p2"), load(root, "p3")
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in p3.values():
        f = fam[family(d["name"])]
        f["launches"] += 1
        f["ns"] += d["ns"]
        for k in ("GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES"):
            f[k] += d.get(k, 0.0)
    for src, key, mul in ((p1, "FETCH_SIZE", 2048.0), (p2, "WRITE_SIZE", 1024.0)):
        for d in src.values():
            f = fam[family(d["name"])]
            f[key] += d.get(key, 0.0) * mul
            f[key + "_ns"] += d["ns"]
    tot_ns = sum(f["ns"] for f in fam.values())
    rows = {}
    for name, f in sorted(fam.items(), key=lambda kv: -kv[1]["ns"]):
        cyc = f["GRBM_GUI_ACTIVE"] / 8.0
        util = f["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * cyc) if cyc else None
        clk = cyc / f["ns"] if f["ns"] else None
        fetch_gbs = f["FETCH_SIZE"] / f["FETCH_SIZE_ns"] if f.get("FETCH_SIZE_ns") else None
        write_gbs = f["WRITE_SIZE"] / f["WRITE_SIZE_ns"] if f.get("WRITE_SIZE_ns") else None
        rows[name] = dict(
            launches_per_step=round(f["launches"] / STEPS, 1), ms_per_step=round(f["ns"] / STEPS / 1e6, 3),
            share_of_serialized_step=round(f["ns"] / tot_ns, 4),
            clock_ghz=round(clk, 3) if clk else None,
            mfma_util=round(util, 4) if util is not None else None,
            mfma_util_of_peak_at_2p4ghz=round(util * clk / PEAK_CLK, 4) if util is not None and clk else None,
            sq_busy_per_cycle=round(f["SQ_BUSY_CYCLES"] / cyc, 3) if cyc else None,
            wave_cycles_per_cycle=round(f["SQ_WAVE_CYCLES"] / cyc, 2) if cyc else None,
            fetch_gb_per_step=round(f["FETCH_SIZE"] / STEPS / 1e9, 3), write_gb_per_step=round(f["WRITE_SIZE"] / STEPS / 1e9, 3),
            hbm_gbs=round((fetch_gbs or 0) + (write_gbs or 0), 1),
            hbm_frac_of_8tbs=round(((fetch_gbs or 0) + (write_gbs or 0)) / 8000.0, 4))
    json.dump({"note": __doc__.strip().split("\n\n")[0], "method": __doc__.strip().split("\n\n", 2)[2],
               "serialized_step_ms": round(tot_ns / STEPS / 1e6, 2), "families": rows}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
