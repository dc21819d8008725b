"""A/B: partition the CUs between the c1 step's two chains with HIP CU masks.

The c1 step is throughput-bound with both chains busy: the teacher forward on the
main stream, the student's forward / backward / AdamW on the module's student stream and the
weight-gradient lane. Each kernel spreads over all 256 CUs, so the chains only overlap in each
other's tails. This measures, in one process on one box, the same model and batches under:
  product      the module's own streams (student + lane at high priority)
  plain        student + lane on unmasked normal-priority streams (the control for the masked arms,
               which hipExtStreamCreateWithCUMask creates at normal priority)
  stu<f>       student + lane masked to a fraction f of every 32-CU word, main unmasked
  split<f>     student + lane on f, the main (teacher) stream on the complement
    python tools/ab_cumask.py [--steps 10 --warmup 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def masked_stream(torch, dev, bits_per_word: int, complement: bool = False, words: int = 8):
    """a normal-priority stream limited to the low `bits_per_word` CUs of every 32-CU mask word
    (or to the others with complement); bits_per_word 32 = unmasked"""
    hip = ctypes.CDLL("libamdhip64.so")
    lo = (1 << bits_per_word) - 1 if bits_per_word < 32 else 0xFFFFFFFF
    w = (~lo & 0xFFFFFFFF) if complement else lo
    mask = (ctypes.c_uint32 * words)(*([w] * words))
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(s.value, device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m, opt = bench.build(bench.CONFIGS["c1"], dev)
    batches = [synthetic_batch(4, dev, L=1536, seed=j) for j in range(2)]
    own = (m._stu_stream, m.student_model.wlane.stream)

    def set_streams(stu, lane):
        m._stu_stream = m._opt_stream = m._bwd_stream = stu
        m.student_model.wlane.stream = lane

    def run(main_stream):
        torch.cuda.synchronize()
        torch.cuda.set_stream(main_stream)

        def step(i):
            loss = m.training_step(batches[i % 2], i)
            loss.backward()
            opt.step()
            opt.zero_grad()
            return loss

        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(a.warmup + i)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return 4 * a.steps / dt, dt / a.steps * 1e3

    plain_main = torch.cuda.Stream(device=dev)
    arms = [("product", lambda: (own, plain_main))]
    arms.append(("plain", lambda: ((torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)), plain_main)))
    for bits in (16, 12, 20):
        arms.append((f"stu{bits}/32", lambda b=bits: ((masked_stream(torch, dev, b), masked_stream(torch, dev, b)),
                                                     plain_main)))
        arms.append((f"split{bits}/32", lambda b=bits: ((masked_stream(torch, dev, b), masked_stream(torch, dev, b)),
                                                       masked_stream(torch, dev, b, complement=True))))
    arms.append(("product_again", lambda: (own, plain_main)))
    for name, mk in arms:
        (stu, lane), main_s = mk()
        set_streams(stu, lane)
        sps, ms = run(main_s)
        print(json.dumps(dict(arm=name, samples_per_s=round(sps, 3), ms_per_step=round(ms, 2))), flush=True)
    set_streams(*own)


if __name__ == "__main__":
    main()
