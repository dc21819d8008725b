"""KD training-step throughput on MI355X (BASELINE.json metric), one JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c4] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step = one `training_step(batch)` + `loss.backward()` + `optimizer.step()` +
`zero_grad()` of the drop-in KD module: 7B RGB teacher forward, 0.5B depth student
forward, fused KD-loss forward+backward, student backward, bucketed RCCL gradient
all-reduce (N > 1) and fused AdamW, on synthetic 336x336 inputs (random pixels, random
token ids) already resident in HBM and random-init weights of the real
architectures (no checkpoints are reachable offline).

Configs (BASELINE.json): c1 = logit-based LoCa (T=1) bs 4 per GPU [default];
c2 = feature-based (NT-Xent + KL) bs 8 per GPU; c3 = double-trouble phase 2 (LoCa, ViT
frozen) bs 8 per GPU; c4 = double-trouble phase 3 bs 8 per GPU (bf16 teacher).
Per-GPU work is fixed as N grows (weak scaling); value = samples of all ranks / max time.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

PEAK_BF16_TFLOPS = 2500.0      # dense bf16 MFMA peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0

CONFIGS = {
    "c1": dict(kind="lb", phase=0, batch=4, desc="logit-based KD (LoCa, T=1), 7B->0.5B, 336x336"),
    "c2": dict(kind="fb", phase=0, batch=8, desc="feature-based KD (NT-Xent + KL), 7B->0.5B, 336x336"),
    "c3": dict(kind="dt", phase=2, batch=8, desc="double-trouble phase 2 (LoCa + CE, ViT frozen)"),
    "c4": dict(kind="dt", phase=3, batch=8, desc="double-trouble phase 3 (0.8 LoCa + CE)"),
}

# algorithmic FLOPs per sample, L = 1536, 2 tiles
def step_tflops_per_sample(kind: str, phase: int) -> float:
    vit = 2 * 1458 * 395.8e6 + 4 * 2 * 729 ** 2 * 1152 * 26 + 2 * 1458 * 0.677e6
    L = 1536
    t_lm = 2 * L * 7070.6e6 + 2 * L * L * 3584 * 28
    s_lm = 2 * L * 494.0e6 + 2 * L * L * 896 * 24
    proj_t = 2 * 1458 * (1152 * 3584 + 3584 * 3584)
    proj_s = 2 * 1458 * (1152 * 896 + 896 * 896)
    teacher = vit + proj_t + t_lm
    s_fwd = vit + proj_s + s_lm
    if kind == "dt" and phase == 2:      # ViT frozen: no ViT backward at all
        s_bwd = 2 * (proj_s + s_lm)
    elif kind == "dt" and phase == 1:    # LM frozen: dgrad only through the LM
        s_bwd = 2 * (vit + proj_s) + (s_lm)
    else:
        s_bwd = 2 * s_fwd
    return (teacher + s_fwd + s_bwd) / 1e12


def build(cfg, dev):
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    S, T = "llava-hf/llava-onevision-qwen2-0.5b-ov-hf", "llava-hf/llava-onevision-qwen2-7b-ov-hf"
    if cfg["kind"] == "lb":
        m = K.LogitBasedKD(S, T)
    elif cfg["kind"] == "fb":
        m = K.FeatureBasedKD(S, T)
    else:
        m = K.OnlineKnowledgeDistillationLLavaOneVision(S, T, phase=cfg["phase"])
        if cfg["phase"] == 2:
            m.freeze_student_vision_layers()
        if cfg["phase"] == 1:
            m.freeze_student_language_layers()
    opts = m.configure_optimizers()
    opt = opts[0][0] if isinstance(opts, tuple) or isinstance(opts, list) else opts
    return m, opt


def cpu_baseline(kind: str, phase: int, threads: int):
    """Oracle (CPU fp32 restatement, `port`) KD step at bs=1, L=1536: full-width teacher and
    student at depth 1 and 3 of every tower (depth 1 timed twice, after and before the
    depth-3 run, min taken: the first run pays allocator/thread-pool warm-up), extrapolated
    to 28/26 + 24/26 layers by the per-layer FLOP share of the depth 1 -> 3 delta (a
    bounded ~40 s sample of the same workload)."""
    import torch
    from oracle.model import OracleLlava, kd_step_losses
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (
        STUDENT_05B, TEACHER_7B, param_specs)
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    from dataclasses import replace
    torch.set_num_threads(threads)
    batch = synthetic_batch(1, "cpu", L=1536, seed=0, pixel_dtype=torch.float32, cpu_rng=True)

    def weights(cfg, seed):
        g = torch.Generator().manual_seed(seed)
        sd = {}
        for s in param_specs(cfg):
            shape = s.ckpt_shape or s.shape
            if s.init == "ones":
                sd[s.name] = torch.ones(shape)
            elif s.init == "zeros":
                sd[s.name] = torch.zeros(shape)
            else:
                sd[s.name] = torch.empty(shape).normal_(0, 0.02, generator=g)
        return sd

    times = {}
    for d in (1, 3, 1):
        tc = replace(TEACHER_7B, vision=replace(TEACHER_7B.vision, layers=d), text=replace(TEACHER_7B.text, layers=d))
        sc = replace(STUDENT_05B, vision=replace(STUDENT_05B.vision, layers=d), text=replace(STUDENT_05B.text, layers=d))
        tsd, ssd = weights(tc, 1), weights(sc, 2)
        train_vision = not (kind == "dt" and phase == 2)
        for k, v in ssd.items():
            v.requires_grad_(train_vision or not k.startswith("vision"))
        teacher, student = OracleLlava(tsd, tc), OracleLlava(ssd, sc)
        t0 = time.perf_counter()
        total, _ = kd_step_losses(kind, teacher, student, batch, phase=phase)
        total.backward()
        times[d] = min(times.get(d, 1e30), time.perf_counter() - t0)
        del tsd, ssd, teacher, student, total
    # per-layer FLOP shares (fwd teacher, fwd+bwd student), L = 1536
    L, NV = 1536, 1458
    vit_layer = 2 * NV * (4 * 1152 ** 2 + 2 * 1152 * 4304) + 4 * 2 * 729 ** 2 * 1152
    t_layer = 2 * L * (2 * 3584 ** 2 + 2 * 3584 * 512 + 3 * 3584 * 18944) + 2 * L * L * 3584
    s_layer = 3 * (2 * L * (2 * 896 ** 2 + 2 * 896 * 128 + 3 * 896 * 4864) + 2 * L * L * 896)
    s_vit = (3 if not (kind == "dt" and phase == 2) else 1) * vit_layer
    parts = dict(t_vit=vit_layer, t_lm=t_layer, s_vit=s_vit, s_lm=s_layer)
    tot = sum(parts.values())
    delta = max((times[3] - times[1]) / 2, 1e-6)   # one layer of every tower
    extra = {"t_vit": 25, "t_lm": 27, "s_vit": 25, "s_lm": 23}
    t_full = times[1] + sum(delta * parts[k] / tot * extra[k] for k in parts)
    return dict(value=round(1.0 / t_full, 5), unit="samples/s", cores=threads, kind="port",
                sample=(f"oracle (CPU fp32 torch restatement) KD step bs=1 L=1536, measured at depth 1 "
                        f"({times[1]:.2f} s, min of 2) and 3 ({times[3]:.2f} s) of every tower, extrapolated to the "
                        f"full 28/26 + 24/26 layers by per-layer FLOP share: {t_full:.1f} s/sample"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c1", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timer", action="store_true", help="skip the serialized roofline pass (per-GEMM HIP events)")
    ap.add_argument("--prefetch", action="store_true",
                    help="run the next step's teacher forward one step ahead on its own stream (measured: no gain, "
                         "the step is GPU-throughput-bound)")
    ap.add_argument("--serial", action="store_true",
                    help="student forward on the main stream (no overlap with the teacher forward)")
    ap.add_argument("--shapes", default=None, help="write the per-shape GEMM timing table (JSON) to this path")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    cfg = CONFIGS[a.config]
    B = a.batch or cfg["batch"]
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    m, opt = build(cfg, dev)
    m.concurrent_student = not a.serial
    # two synthetic batches, alternated, so every step's teacher forward is a fresh one
    batches = [synthetic_batch(B, dev, L=1536, seed=rank * 2 + j) for j in range(2)]
    prefetch = [a.prefetch and not a.serial]

    def step(i):
        loss = m.training_step(batches[i % 2], i)
        loss.backward()
        if prefetch[0]:   # the next step's teacher forward, beside this step's backward + AdamW
            m.prefetch_teacher(batches[(i + 1) % 2])
        opt.step()
        opt.zero_grad()
        return loss

    # the step's main stream at the same high priority as its side streams (the teacher
    # prefetch stream stays at normal priority)
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import STREAM_PRIORITY_HIGH
    hp = torch.cuda.Stream(device=dev, priority=STREAM_PRIORITY_HIGH)
    hp.wait_stream(torch.cuda.current_stream())
    torch.cuda.set_stream(hp)
    for i in range(a.warmup):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(a.warmup + i)
    host_dt = time.perf_counter() - t0   # host enqueue time of the K steps (~dt: launch-bound)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # roofline pass (untimed): two steps with the student forward serialized behind the
    # teacher forward, every GEMM bracketed by HIP events on its launch stream, so a
    # kernel's duration is its own and not shared with a concurrent stream
    if not a.no_timer:
        m.concurrent_student = False
        prefetch[0] = False
        m._prefetched = None   # the roofline steps run every teacher GEMM inline, on the main stream
        ops.TIMER.reset()
        ops.TIMER.enabled = True
        for i in range(2):
            step(a.warmup + a.steps + i)
        torch.cuda.synchronize()
        ops.TIMER.enabled = False
        m.concurrent_student = not a.serial
        prefetch[0] = a.prefetch and not a.serial
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    samples = world * B * a.steps
    value = samples / dt
    tf_sample = step_tflops_per_sample(cfg["kind"], cfg["phase"])
    roof = None
    br = {}
    for kind in ("gemm_kk_swiglu", "gemm_kk", "gemm_kn", "gemm_nn"):
        s = ops.TIMER.summary(kind)
        if s:
            br[kind] = dict(launches=s["launches"], avg_us=round(s["avg_ms"] * 1e3, 2),
                            tflops=round(s["flops"] / (s["total_ms"] * 1e-3) / 1e12, 1),
                            share_of_step=round(s["total_ms"] / 2 * 1e-3 / (dt / a.steps), 3))
    if a.shapes and rank == 0 and ops.TIMER.records:
        with open(a.shapes, "w") as f:
            json.dump(ops.TIMER.by_shape(top=200), f, indent=1)
    # the roofline kernel: the fused gate|up + SwiGLU GEMM (k_gemm8<K-major,K-major> SwiGLU build,
    # one launch per call, 28 + 24 calls per step, ~40% of the step's GEMM time) -- a kernel of
    # its own, so the rocprofv3 kernel trace's average for it is directly comparable
    fwd = ops.TIMER.summary("gemm_kk_swiglu")
    traffic = None   # PMC HBM bytes per forward-GEMM launch (tools/pmc_bench.sh, committed under profiles/)
    tpath = REPO / "profiles" / "r01" / "pmc_traffic.json"
    if tpath.exists():
        fg = json.load(open(tpath)).get("roofline_kernel")
        if fg:
            traffic = round(fg["traffic_bytes"])
    if fwd:
        ach = fwd["flops"] / (fwd["total_ms"] * 1e-3) / 1e12
        roof = dict(bound="mfma", kernel="k_gemm8<false, false, 4> (fused gate|up GEMM + SwiGLU epilogue of every "
                                           "teacher and student MLP, bf16)",
                    achieved=round(ach, 1), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s", frac=round(ach / PEAK_BF16_TFLOPS, 4),
                    traffic=traffic, traffic_unit="bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                                                   "profiles/r01/pmc_traffic.json)",
                    flops_per_launch=round(fwd["flops_per_launch"] / 1e9, 2),
                    avg_launch_us=round(fwd["avg_ms"] * 1e3, 2),
                    measured="HIP events on the launch stream over 2 serialized steps after the timed region "
                             "(bench.py --serial under rocprofv3 gives the matching kernel trace)")
    out = {
        "metric": "KD samples/sec/step (7B->0.5B, 336x336)",
        "value": round(value, 4),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random 336x336 pixels, random token ids; random-init weights of the real architectures)",
        "config": {"workload": f"{a.config}: {cfg['desc']}", "model": "llava-onevision-qwen2-7b (teacher) -> 0.5b (student)",
                   "global_batch": world * B, "per_gpu_batch": B, "seq_len": 1536, "image": "336x336 (2 tiles, 1485 tokens)",
                   "parallelism": f"dp{world}",
                   "teacher_prefetch": bool(a.prefetch and not a.serial)},
        "mfu": round(value * tf_sample / world / PEAK_BF16_TFLOPS, 4),
        "host_enqueue_ms_per_step": round(host_dt * 1e3 / a.steps, 2),
        "tflop_per_sample": round(tf_sample, 2),
        "loss": round(float(loss.item()), 5),
        "roofline": roof,
        "gemm_breakdown": br,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        try:
            out["cpu_baseline"] = cpu_baseline(cfg["kind"], cfg["phase"], threads)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
