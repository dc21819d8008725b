"""Host time of each call of a c1 bench step (after warmup), to see where the host waits:
    python tools/host_phases.py [--config c1] [--steps 4]
Prints per step: training_step / backward / opt.step / zero_grad host ms, and the GPU time of
the step (HIP events on the main stream)."""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--idle", action="store_true", help="synchronize before each step (host cost on an idle GPU)")
    a = ap.parse_args()
    import torch
    import bench
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import STREAM_PRIORITY_HIGH
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[a.config]
    m, opt = bench.build(cfg, dev, teacher_fp8=bool(cfg.get("teacher_fp8")))
    batches = [synthetic_batch(cfg["batch"], dev, L=1536, seed=j) for j in range(2)]
    hp = torch.cuda.Stream(device=dev, priority=int(__import__("os").environ.get("KD_MAIN_STREAM_PRIORITY", "0")))
    hp.wait_stream(torch.cuda.current_stream())
    torch.cuda.set_stream(hp)
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops as OPS
    tm = {}

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def g(*args, **kw):
            t0 = time.perf_counter()
            r = f(*args, **kw)
            tm[key] = tm.get(key, 0.0) + (time.perf_counter() - t0) * 1e3
            return r
        setattr(obj, name, g)
    wrap(m._errors, "check", "errors.check")
    wrap(m._errors, "record", "errors.record")
    if m.teacher_model is not None:
        wrap(m.teacher_model, "forward", "teacher.forward")
    wrap(m.student_model, "forward", "student.forward")
    wrap(m.student_model, "backward", "student.backward")
    wrap(m.student_model.wlane, "run", "wlane.run")
    wrap(OPS, "kd_loss_fwd_bwd", "ops.kd_loss")
    wrap(OPS, "gemm", "ops.gemm")
    wrap(m, "_check_errors", "m._check_errors")
    # GPU-side markers (elapsed ms from the step's first event): when the main stream reaches
    # the teacher forward, when the teacher forward and the loss end, when the backward ends
    marks = {}

    hmarks = {}
    t_host0 = [None]

    def mark(name, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream or torch.cuda.current_stream())
        marks.setdefault(name, []).append(e)
        now = time.perf_counter()
        if t_host0[0] is None:
            t_host0[0] = now
        hmarks.setdefault(name, []).append(round((now - t_host0[0]) * 1e3, 1))

    tf = m.teacher_model.forward

    def tf_marked(*args, **kw):
        mark("teacher_start")
        r = tf(*args, **kw)
        mark("teacher_end")
        return r
    m.teacher_model.forward = tf_marked
    bw = m._backward

    def bw_marked(g):
        mark("bwd_enqueued_main")
        r = bw(g)
        mark("bwd_end", m._bwd_stream)
        return r
    m._backward = bw_marked
    sf = m.student_model.forward

    def sf_marked(*args, **kw):
        mark("student_start")
        r = sf(*args, **kw)
        mark("student_end")
        return r
    m.student_model.forward = sf_marked
    ad = OPS.adamw

    def ad_marked(*args, **kw):
        mark("adamw_start")
        r = ad(*args, **kw)
        mark("adamw_end")
        return r
    OPS.adamw = ad_marked
    for i in range(2 + a.steps):
        if a.idle:
            torch.cuda.synchronize()
        tm.clear()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t = [time.perf_counter()]
        loss = m.training_step(batches[i % 2], i)
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        opt.zero_grad()
        t.append(time.perf_counter())
        e1.record()
        d = [round((t[k + 1] - t[k]) * 1e3, 2) for k in range(4)]
        print(f"step {i}: host ms training_step {d[0]} backward {d[1]} opt.step {d[2]} zero_grad {d[3]} "
              f"(total {round((t[-1] - t[0]) * 1e3, 1)}) inner {dict((k, round(v, 2)) for k, v in tm.items())}", flush=True)
    torch.cuda.synchronize()
    base = marks["teacher_start"][0]
    for k in range(len(marks["teacher_start"])):
        row = {n: round(base.elapsed_time(v[k]), 1) for n, v in marks.items() if k < len(v)}
        print("gpu marks step", k, row)
        print("host marks step", k, {n: v[k] for n, v in hmarks.items() if k < len(v)})


if __name__ == "__main__":
    main()
