"""A/B of step-level scheduling knobs of the c1 step, in one process on one box (interleaved arms):
  product        the module as shipped (student chain + weight-gradient lane + main stream)
  lane_serial    the student's weight gradients on the student chain's stream (no third stream)
  stats_late     the student row statistics of the KD loss computed on the main stream with the
                 teacher's (kd_module.student_stats_early = False)
    python tools/ab_step_knobs.py [--steps 10 --warmup 3 --rounds 2]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bench
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m, opt = bench.build(bench.CONFIGS["c1"], dev)
    batches = [synthetic_batch(4, dev, L=1536, seed=j) for j in range(2)]
    torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=0))

    def run():
        def step(i):
            loss = m.training_step(batches[i % 2], i)
            loss.backward()
            opt.step()
            opt.zero_grad()

        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(a.warmup + i)
        torch.cuda.synchronize()
        return 4 * a.steps / (time.perf_counter() - t0)

    def setk(lane_serial=False, stats_early=True):
        torch.cuda.synchronize()
        m.student_model.wlane.serial = lane_serial
        m.student_stats_early = stats_early

    arms = [("product", {}), ("lane_serial", dict(lane_serial=True)), ("stats_late", dict(stats_early=False))]
    for r in range(a.rounds):
        for name, kw in arms:
            setk(**kw)
            print(json.dumps(dict(round=r, arm=name, samples_per_s=round(run(), 3))), flush=True)
    setk()


if __name__ == "__main__":
    main()
