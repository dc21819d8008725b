# bf16 vs fp32 drift of the CPU oracle teacher (real widths, random N(0,0.02) weights) by depth
import sys, json, torch
sys.path.insert(0, '/root/repo')
from dataclasses import replace
from oracle.model import OracleLlava
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import TEACHER_7B, param_specs
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
torch.set_num_threads(8)
b = synthetic_batch(1, "cpu", L=1536, seed=0, pixel_dtype=torch.float32, cpu_rng=True)
for d in [int(x) for x in sys.argv[1].split(",")]:
    cfg = replace(TEACHER_7B, vision=replace(TEACHER_7B.vision, layers=min(d, 26)), text=replace(TEACHER_7B.text, layers=d))
    g = torch.Generator().manual_seed(1)
    sd = {}
    for s in param_specs(cfg):
        shape = s.ckpt_shape or s.shape
        sd[s.name] = torch.ones(shape) if s.init == "ones" else torch.zeros(shape) if s.init == "zeros" else torch.empty(shape).normal_(0, 0.02, generator=g).bfloat16().float()
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        w = {k: v.to(dt) for k, v in sd.items()}
        with torch.no_grad():
            lg, _ = OracleLlava(w, cfg)(b["rgb_input_ids"], b["rgb_pixel_values"].to(dt), b["image_sizes"])
        res[dt] = lg.float()
    a, c = res[torch.bfloat16], res[torch.float32]
    print(json.dumps(dict(depth=d, bf16_vs_fp32_logits_rel_l2=float((a - c).norm() / c.norm()), cosine=float((a*c).sum()/(a.norm()*c.norm())))), flush=True)
