"""fp8 (OCP e4m3) path of the fp8 teacher (BASELINE config c4): the row quantiser against
torch's float8_e4m3fn cast (scales within 1 ulp — the two divisions may round apart — and
codes equal except at those rounding boundaries, where they are adjacent), and the fp8 MFMA GEMM against a torch fp32 product of
the dequantised operands (e4m3 x e4m3 products are exact in fp32; only the summation order
and the bf16 output rounding differ):  |out - ref| <= 2^-7 |ref| + 1e-4 rms(ref)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops
    return ops


def _quant_ref(x):
    """The quantiser's definition in torch: scale = amax / 448, q = e4m3(clamp(x * 448 / amax))."""
    xf = x.float()
    amax = xf.abs().amax(1)
    inv = torch.where(amax > 0, torch.tensor(448.0, device=x.device) / amax, torch.ones_like(amax))
    q = (xf * inv[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))


def _deq(q, s):
    return q.view(torch.float8_e4m3fn).float() * s[:, None]


@pytest.mark.parametrize("R,K", [(1, 16), (37, 1152), (300, 3584), (8, 18944)])
def test_quant_rows_matches_torch_e4m3(R, K, dev):
    ops = _ops()
    g = torch.Generator(device=dev).manual_seed(R + K)
    x = (torch.randn(R, K, generator=g, device=dev) * 3).to(torch.bfloat16)
    x[0, :5] = torch.tensor([0.0, -0.0, 1e-8, -5e-6, 1e-30], device=dev).to(torch.bfloat16)   # tiny values
    if R > 2:
        x[2] = 0   # an all-zero row: scale 1
    q, s = ops.quant_rows_fp8(x)
    qr, sr = _quant_ref(x)
    torch.cuda.synchronize()
    assert torch.allclose(s, sr, rtol=2.5e-7, atol=0)
    diff = (q.view(torch.float8_e4m3fn).float() - qr.view(torch.float8_e4m3fn).float()).abs()
    ulp = qr.view(torch.float8_e4m3fn).float().abs().clamp_min(2.0 ** -6) * 2.0 ** -3   # e4m3 step
    mism = int((q != qr).sum())
    assert bool((diff <= ulp * 1.001).all()) and mism <= max(1, q.numel() // 1000), f"{mism} of {q.numel()} differ"


def _check(out, ref, what, scale=None):
    ref = ref.float()
    err = (out.float() - ref).abs()
    tol = 2.0 ** -7 * (ref.abs() if scale is None else scale) + 1e-4 * ref.pow(2).mean().sqrt()
    bad = int((err > tol).sum())
    assert bad == 0, f"{what}: {bad} of {err.numel()} out of tolerance, max err {err.max().item():.3e}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 160), (512, 1024, 3584), (37, 264, 48)])
def test_gemm_fp8_matches_dequantised_product(M, N, K, dev):
    ops = _ops()
    g = torch.Generator(device=dev).manual_seed(M * 7 + N)
    a = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.05).to(torch.bfloat16)
    qa, sa = ops.quant_rows_fp8(a)
    qb, sb = ops.quant_rows_fp8(w)
    out = ops.gemm_fp8(qa, sa, qb, sb)
    ref = _deq(qa, sa) @ _deq(qb, sb).t()
    _check(out, ref, "plain")
    # epilogue: alpha, bias, gelu, residual (the output rounds gelu(pre) to bf16 before the
    # residual add: the tolerance is taken on the magnitude of the two summands)
    bias = torch.randn(N, generator=g, device=dev).to(torch.bfloat16)
    res = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16)
    out2 = ops.gemm_fp8(qa, sa, qb, sb, bias=bias, act="gelu_tanh", residual=res, alpha=0.5)
    act = torch.nn.functional.gelu(0.5 * ref + bias.float(), approximate="tanh")
    _check(out2, act.bfloat16().float() + res.float(), "epilogue", scale=2 * (act.abs() + res.float().abs()))


def test_gemm_fp8_swiglu(dev):
    ops = _ops()
    M, I, K = 600, 384, 512
    g = torch.Generator(device=dev).manual_seed(5)
    a = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(2 * I, K, generator=g, device=dev) * 0.05).to(torch.bfloat16)
    qa, sa = ops.quant_rows_fp8(a)
    qb, sb = ops.quant_rows_fp8(w)
    aux = torch.empty(M, 2 * I, dtype=torch.bfloat16, device=dev)
    h = ops.gemm_fp8(qa, sa, qb, sb, act="swiglu", aux=aux)
    v = _deq(qa, sa) @ _deq(qb, sb).t()
    _check(aux, v, "gate|up")
    gu = v.bfloat16().float()
    # gate / up are rounded to bf16 from the kernel's own fp32 sums (one bf16 ulp apart from
    # the reference's where a sum straddles a rounding boundary): 2 ulps of the product
    sw = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
    _check(h, sw, "swiglu", scale=2 * sw.abs())


def test_gemm_fp8_teacher_shape_sampled(dev):
    """c4's largest teacher GEMM shape class (6144 x 3584 x 18944, down_proj) on sampled rows."""
    ops = _ops()
    M, N, K = 6144, 3584, 18944
    g = torch.Generator(device=dev).manual_seed(9)
    a = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    qa, sa = ops.quant_rows_fp8(a)
    qb, sb = ops.quant_rows_fp8(w)
    out = ops.gemm_fp8(qa, sa, qb, sb)
    rows = torch.tensor([0, 1, 255, 256, 3000, 6143], device=dev)
    ref = _deq(qa[rows], sa[rows]) @ _deq(qb, sb).t()
    _check(out[rows], ref, "rows")


def test_fp8_teacher_end_to_end_tiny(dev):
    """LogitBasedKD with every teacher linear on the fp8 path vs the same module with the bf16
    teacher, same weights and batch (tiny widths, 2 layers): the student side is untouched
    (student CE bit-equal), the teacher logits stay within rel-L2 0.15 / cosine 0.99 of the
    bf16 teacher's and the KD term within 0.15 relative.  The full-width depth tolerance is
    test_fp8_teacher_depth8_real_widths."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
    from model_fixtures import batch, load
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    meta, _ = load("lb")
    b = batch(meta, dev)
    out = {}
    for fp8 in (False, True):
        m = K.LogitBasedKD("tiny-student", "tiny-teacher", teacher_fp8=fp8)
        m.keep_logits = True
        total = m.forward(b)
        torch.cuda.synchronize()
        s3, t3 = m.last_logits
        out[fp8] = (total.item(), m.last_terms.tolist(), t3.float().clone(), s3.float().clone())
    (_, terms_b, t_b, s_b), (_, terms_f, t_f, s_f) = out[False], out[True]
    assert torch.equal(s_b, s_f) and terms_b[1] == terms_f[1]          # student untouched
    rel = float((t_f - t_b).norm() / t_b.norm())
    cos = float((t_f * t_b).sum() / (t_f.norm() * t_b.norm()))
    kd_rel = abs(terms_f[0] - terms_b[0]) / abs(terms_b[0])
    print(f"fp8 teacher: logits rel-L2 {rel:.4f} cosine {cos:.5f}; KD term {terms_f[0]:.6g} vs {terms_b[0]:.6g} "
          f"(rel {kd_rel:.4f}); teacher CE {terms_f[2]:.6g} vs {terms_b[2]:.6g}")
    assert 0 < rel <= 0.15 and cos >= 0.99, (rel, cos)
    assert kd_rel <= 0.15, (terms_f[0], terms_b[0])


@pytest.mark.parametrize("families,max_rel,min_cos", [("lm_mlp", 0.18, 0.98), ("all", 0.32, 0.95)])
def test_fp8_teacher_depth8_real_widths(families, max_rel, min_cos, dev):
    """The 7B teacher at its real widths, 8 Qwen2 + 8 SigLIP layers, one 336x336 sample: the
    fp8 policy's logits against the bf16 teacher's (same weights).  Stated tolerances (DESIGN
    §4; measured 0.155 / 0.988 for lm_mlp — BASELINE c4's default — and 0.284 / 0.960 for all,
    profiles/r03/fp8_depth_policies.json).  e4m3 costs ~3.7 % rel-L2 per GEMM output whatever
    the scaling and the errors add in quadrature along the forward, so the bound grows with
    depth (full depth: 0.249 / 0.969 and 0.478 / 0.886)."""
    from dataclasses import replace
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (TEACHER_7B,
                                                                                                   LlavaOnevisionModel)
    cfg = replace(TEACHER_7B, vision=replace(TEACHER_7B.vision, layers=8), text=replace(TEACHER_7B.text, layers=8))
    t = LlavaOnevisionModel(cfg, dev, trainable=False, seed=1)
    b = synthetic_batch(1, dev, L=1536, seed=0)
    out = {}
    for fam in (None, families):
        if fam:
            t.enable_fp8(fam)
        with torch.no_grad():
            f = t.forward(b["rgb_input_ids"], b["rgb_pixel_values"], b["image_sizes"], want_logits=True)
        torch.cuda.synchronize()
        out[fam] = f["logits"].float()
    lb, lf = out[None], out[families]
    rel = float((lf - lb).norm() / lb.norm())
    cos = float((lf * lb).sum() / (lf.norm() * lb.norm()))
    print(f"fp8 {families} depth 8: logits rel-L2 {rel:.4f} cosine {cos:.5f}")
    assert 0 < rel <= max_rel and cos >= min_cos, (rel, cos)


@pytest.mark.parametrize("name,families", [("real_dt2", "lm_mlp"), ("real_lb", "lm_mlp"), ("real_dt2", "all"),
                                           ("real_dt3", "lm_mlp")])
def test_fp8_teacher_real_widths_vs_reference(name, families, dev):
    """The fp8 teacher against the REFERENCE, not against the bf16 teacher: the drop-in module at
    the real widths (2 layers per tower; SigLIP 1152 x hd 72, Qwen2-7B 3584/18944 GQA 28/4,
    Qwen2-0.5B 896/4864) with the teacher's linears of `families` on the e4m3 path, one
    training_step on the fixture's batch, each loss term against the reference's own fp32
    forward()/training_step (tests/golden/model_real_*.npz; real_dt3 is BASELINE c4's own phase,
    DT phase 3).  The student side does not see the
    teacher's precision: student CE at the north-star tolerance.  The teacher-dependent terms
    carry the e4m3 error (~3.7 % rel-L2 per GEMM output): stated tolerance of BASELINE c4's fp8
    teacher -- KD term within 1 %, teacher CE within 1 %, total within 1 %."""
    from step_parity import module
    from model_fixtures import EVERY_KIND, batch, load, module_names
    meta, exp = load(name)
    kind, phase = EVERY_KIND[name]
    m = module(kind, phase, module_names(meta))
    m.teacher_model.enable_fp8(families)
    m.teacher_fp8 = families
    loss = m.training_step(batch(meta, dev), 0)
    torch.cuda.synchronize()
    assert int(m.student_model.err.item()) == 0
    kd, ce, tce, _ = m.last_terms.tolist()
    ref = {k: float(exp[k]) for k in ("kd_term", "student_ce", "teacher_ce", "total")}
    d = {"kd_term": abs(kd - ref["kd_term"]) / abs(ref["kd_term"]),
         "teacher_ce": abs(tce - ref["teacher_ce"]) / abs(ref["teacher_ce"]),
         "total": abs(loss.item() - ref["total"]) / abs(ref["total"])}
    print(f"fp8 {families} {name}: rel vs reference {d}; student CE {ce:.6g} vs {ref['student_ce']:.6g}")
    assert abs(ce - ref["student_ce"]) <= 1e-4 + 1e-3 * abs(ref["student_ce"])
    assert d["kd_term"] <= 1e-2 and d["teacher_ce"] <= 1e-2 and d["total"] <= 1e-2, d


@pytest.mark.timeout(600)
def test_c4_fp8_kd_term_within_stated_tolerance(dev):
    """BASELINE config c4 at its full per-GPU size (DT phase 3, LoCa T = 0.8, bs 8, the fp8 lm_mlp
    teacher): bench.py's fp8_teacher_delta on a fresh step's batch.  The KD term's move against
    the bf16 teacher splits into the change of LoCa's second index (DT:170-171, which decides the
    global klogit column overrides, KAT 1) and the smooth change of the teacher probabilities with
    that index held.  Held: the smooth part within the stated 1.5 % (bench.FP8_KD_TOL; measured +0.81 ...
    +0.89 % with fresh students, +1.11 % after the c4 bench's 13 steps, profiles/r06/fp8_c4*.json and
    bench_c4.json); the split adds up to the kernel's own KD-term move (the oracle's
    arithmetic on the same logits: |rel difference| <= 1e-4).  The flip part (measured -2.6 ...
    +0.9 %) is top-2 index noise of a random-init teacher whose top two logits tie at bf16
    resolution: a rounding-order-only perturbation of the bf16 teacher (its Qwen2 residual stream
    in fp32) moves the term by up to 1.7 % the same way (reported, not held)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    m = K.OnlineKnowledgeDistillationLLavaOneVision("llava-hf/llava-onevision-qwen2-0.5b-ov-hf",
                                                    "llava-hf/llava-onevision-qwen2-7b-ov-hf", phase=3,
                                                    teacher_fp8="lm_mlp")
    r = bench.fp8_teacher_delta(m, synthetic_batch(8, dev, L=1536, seed=0))
    sp = r["kd_split"]
    assert abs(sp["smooth"]) <= bench.FP8_KD_TOL, sp
    assert r["within_tolerance"]
    assert abs(sp["total"] - r["terms"]["kd_term"]["rel"]) <= 1e-4, (sp, r["terms"]["kd_term"])
    assert abs(r["terms"]["teacher_ce"]["rel"]) <= 0.01, r["terms"]["teacher_ce"]
    assert r["terms"]["student_ce"]["rel"] == 0.0     # the student never sees the teacher's precision
    assert r["teacher_logits_cosine"] >= 0.96 and r["teacher_logits_rel_l2"] <= 0.27, r
    assert m.teacher_model.fp8                        # the module is left with its fp8 teacher
