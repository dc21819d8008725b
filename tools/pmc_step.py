"""Per kernel family of the serialized c1 step: time, MFMA utilisation and HBM traffic (north_star:
"rocprof HBM GB/s and MFMA utilisation against gfx950 peak").

    python tools/pmc_step.py <pmc_bench dir> <kernel_trace.csv> > pmc_step.json

Inputs (tools/gpu_round.sh steps prof + pmcstep; every run is `bench.py --serial`, so one kernel at a time):
  kernel_trace.csv   rocprofv3 --kernel-trace of the bench (no counters): each family's WALL time per step
  p1 FETCH_SIZE, p2 WRITE_SIZE, p3 GRBM_GUI_ACTIVE + SQ_WAVE_CYCLES + SQ_BUSY_CYCLES +
  SQ_VALU_MFMA_BUSY_CYCLES   (--pmc passes of a shorter run of the same bench; counters per step)
A run's step count is its number of k_adamw dispatches (one per optimizer step), so both sources are
per step.  Counter-collection passes run slower than the plain trace (measured +40-55 % on the big
GEMMs) and GRBM_GUI_ACTIVE / 8 / wall reads high on short dispatches (MI355X_MICROARCH, DVFS
give-back), so the wall time and the clock are NOT taken from the counter passes:
  mfma_util_vs_peak = MFMA_BUSY per step / (1024 SIMDs x 2.4 GHz x traced wall per step)
      SQ_VALU_MFMA_BUSY_CYCLES counts MFMA pipe cycles summed over the SIMDs (16 per 16x16x32 bf16 MFMA,
      32 per 32x32x16): at 2.4 GHz the 1024 SIMDs deliver the 2.5 PF dense bf16 peak, so this is the
      fraction of that peak the family's MFMAs would take at the peak clock -- for a bf16 GEMM family it
      equals achieved TF/s / 2.5 PF (the fp8 MFMA counts its own cycles, 2x the FLOPs per cycle);
  hbm = (FETCH_SIZE x 2 (gfx950 wide-read correction) + WRITE_SIZE) per step / traced wall per step
      (FETCH_SIZE counts L2 -> fabric bytes, Infinity-Cache hits included: an upper bound of HBM reads).
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import re
import sys

N_SIMD = 1024
PEAK_CLK_GHZ = 2.4


def family(n: str) -> str:
    if "k_gemm8f8" in n:
        return "gemm fp8"
    m = re.search(r"k_gemm(8|3)<(?:\d+, \d+, )?(true|false), (true|false)(?:, (\d+))?", n)
    if m:
        amn, bmn = m.group(2) == "true", m.group(3) == "true"
        exp = int(m.group(4) or 0) if m.group(1) == "8" else 0   # k_gemm3's 5th parameter is its ring depth
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
    if "k_colsum" in n:
        return "bias colsum"
    if "k_embed" in n or "k_image_src" in n or "k_patchify" in n:
        return "embeddings / patchify"
    if "k_qkv" in n or "k_swiglu" in n or "k_act_bwd" in n:
        return "qkv / activation (unfused)"
    if n.startswith("kd::") or "kd::(anonymous" in n or "_ZN2kd" in n:
        return "other kd kernels"
    return "torch (allocator fills, casts)"


def load_pmc(root, pas):
    out = {}
    for f in glob.glob(f"{root}/{pas}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = out.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "t": int(r["Start_Timestamp"])})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # the step window opens at the run's first KD kernel (model construction is not a step)
    t0 = min((v["t"] for v in out.values() if family(v["name"]) != "torch (allocator fills, casts)"), default=0)
    return {k: v for k, v in out.items() if v["t"] >= t0}


def steps_of(names):
    return max(1, sum(1 for n in names if "k_adamw" in n))


def main():
    root, trace = sys.argv[1], sys.argv[2]
    wall = collections.defaultdict(float)
    calls = collections.defaultdict(int)
    tnames = []
    started = False
    for r in sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"])):
        n = r["Kernel_Name"]
        # the run's first KD kernel opens the step window: model construction (weight init) is not a step
        started = started or family(n) not in ("torch (allocator fills, casts)",)
        if not started:
            continue
        tnames.append(n)
        f = family(n)
        wall[f] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        calls[f] += 1
    t_steps = steps_of(tnames)
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    p_steps = {}
    for pas, keys in (("p1", ("FETCH_SIZE",)), ("p2", ("WRITE_SIZE",)),
                      ("p3", ("GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES"))):
        d = load_pmc(root, pas)
        p_steps[pas] = steps_of([v["name"] for v in d.values()])
        for v in d.values():
            for k in keys:
                cnt[family(v["name"])][k] += v.get(k, 0.0) / p_steps[pas]
    tot = sum(wall.values()) / t_steps
    mfma_all = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for c in cnt.values())
    rows = {}
    for f in sorted(wall, key=lambda k: -wall[k]):
        ns = wall[f] / t_steps
        c = cnt.get(f, {})
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        fetch = c.get("FETCH_SIZE", 0.0) * 2048.0   # KB, x2
        write = c.get("WRITE_SIZE", 0.0) * 1024.0
        rows[f] = dict(launches_per_step=round(calls[f] / t_steps, 1), ms_per_step=round(ns / 1e6, 3),
                       share_of_serialized_step=round(ns / 1e6 / (tot / 1e6), 4),
                       mfma_util_vs_peak=round(mfma / (N_SIMD * PEAK_CLK_GHZ * ns), 4) if ns else None,
                       fetch_gb_per_step=round(fetch / 1e9, 3), write_gb_per_step=round(write / 1e9, 3),
                       hbm_gbs=round((fetch + write) / ns, 1) if ns else None,
                       hbm_frac_of_8tbs=round((fetch + write) / ns / 8000.0, 4) if ns else None,
                       sq_busy_per_wave_cycle=round(c["SQ_BUSY_CYCLES"] / c["SQ_WAVE_CYCLES"], 4)
                       if c.get("SQ_WAVE_CYCLES") else None)
    doc = __doc__.strip()
    json.dump({"what": doc.split("\n\n")[0], "method": doc.split("\n\n", 2)[2],
               "steps": {"trace": t_steps, **p_steps}, "serialized_step_ms": round(tot / 1e6, 2),
               "step_mfma_util_vs_peak": round(mfma_all / (N_SIMD * PEAK_CLK_GHZ * tot), 4), "families": rows},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main()
