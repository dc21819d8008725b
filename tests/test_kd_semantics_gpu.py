"""Trainer semantics of the drop-in modules on the GPU: label-range errors surface as the
reference's RuntimeError (DT:166), loss groups / gradient accumulation reproduce the
reference's batch_size=1 x accumulate_grad_batches training (DT1T:70, :155), a 2-rank
data-parallel step equals the single-process step on the union batch, and checkpoints
reload through load_from_checkpoint with the reference's keyword arguments."""
import math
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from model_fixtures import batch, load

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parent.parent


def _K():
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    return K


def _grads(m):
    lo, hi = m._trainable_range()
    return m.student_model.P.grad[lo:hi].double().clone()


def _close_grads(a, b, rel=2e-3):
    cos = float((a @ b) / (a.norm() * b.norm()))
    nr = float(a.norm() / b.norm())
    assert cos >= 0.9999 and abs(nr - 1) <= rel, f"cosine {cos:.6f}, norm ratio {nr:.6f}"


def _attempt(f, raised):
    try:
        f()
    except RuntimeError as e:
        raised.append(str(e))


def test_loca_minus100_label_raises_before_the_update(dev):
    """LoCa gathers at every label: -100 (a pad) is out of bounds (DT:166, SURVEY KAT 2).
    AdamW skips on the step's device error words, so the weights never change; the host
    reports the error once, at the first training_step / optimizer.step after the loss
    kernel has finished (no host wait on the step's path); training then continues."""
    K = _K()
    meta, _ = load("lb")
    m = K.LogitBasedKD("tiny-student", "tiny-teacher")
    (opt,), _ = m.configure_optimizers()
    good = batch(meta, dev)
    b = dict(good)
    b["labels"] = good["labels"].clone()
    b["labels"][1, 37] = -100
    before = m.student_model.P.flat.clone()
    master = m.student_model.P.master.clone()
    raised = []
    m.training_step(b, 0).backward()
    _attempt(opt.step, raised)
    opt.zero_grad()
    torch.cuda.synchronize()
    assert torch.equal(m.student_model.P.flat, before) and torch.equal(m.student_model.P.master, master)
    if not raised:   # the loss kernel has finished now: the next call reports it
        _attempt(lambda: m.training_step(good, 1), raised)
    assert len(raised) == 1, raised
    assert re.search(r"index -100 is out of bounds for dimension 2.*batch 1, position 37", raised[0]), raised
    # reported once; a valid batch trains again
    m.training_step(good, 2).backward()
    opt.step()
    m.check_errors()
    torch.cuda.synchronize()   # AdamW runs on the module's student stream
    assert not torch.equal(m.student_model.P.flat, before)


@pytest.mark.skipif(not hasattr(torch.cuda, "_sleep"), reason="needs torch.cuda._sleep")
def test_error_words_are_sticky_for_queued_steps(dev):
    """A valid step queued behind a rejected one (the host has not seen the error yet)
    does not update the weights either: the state after the report is the state before
    the rejected batch, as after the reference's RuntimeError."""
    K = _K()
    meta, _ = load("lb")
    m = K.LogitBasedKD("tiny-student", "tiny-teacher")
    (opt,), _ = m.configure_optimizers()
    good = batch(meta, dev)
    bad = dict(good)
    bad["labels"] = good["labels"].clone()
    bad["labels"][0, 5] = -100
    torch.cuda.synchronize()
    before = m.student_model.P.flat.clone()
    torch.cuda._sleep(2_000_000_000)   # hold the stream: both steps are queued before either runs
    raised = []
    for i, bt in enumerate((bad, good)):   # a trainer stops at the first reported error
        _attempt(lambda: m.training_step(bt, i).backward(), raised)
        if not raised:
            _attempt(opt.step, raised)
        if raised:
            break
        opt.zero_grad()
    if not raised:
        _attempt(m.check_errors, raised)
    torch.cuda.synchronize()
    assert len(raised) == 1 and "index -100" in raised[0], raised
    assert torch.equal(m.student_model.P.flat, before)


@pytest.mark.skipif(not hasattr(torch.cuda, "_sleep"), reason="needs torch.cuda._sleep")
def test_next_steps_teacher_error_does_not_cancel_this_update(dev):
    """Step t is valid; step t+1's RGB ids carry one image token too few (the teacher's
    masked_scatter size mismatch).  Step t+1's teacher forward runs on the main stream
    beside step t's AdamW (held back here on the student stream), so its error word is
    set before AdamW t runs: AdamW t must still apply (it reads the words as of its own
    loss), AdamW t+1 must not, and the error is reported once."""
    K = _K()
    meta, _ = load("lb")
    good = batch(meta, dev)
    bad = dict(good)
    bad["rgb_input_ids"] = good["rgb_input_ids"].clone()
    img = (bad["rgb_input_ids"][0] == 151646).nonzero()[0, 0]
    bad["rgb_input_ids"][0, img] = 100
    # the expected state: one valid step, fully synchronised
    r = K.LogitBasedKD("tiny-student", "tiny-teacher")
    (ropt,), _ = r.configure_optimizers()
    w0 = r.student_model.P.master.clone()
    r.training_step(good, 0).backward()
    ropt.step()
    r.check_errors()
    torch.cuda.synchronize()
    ref_upd = (r.student_model.P.master - w0).double()
    m = K.LogitBasedKD("tiny-student", "tiny-teacher")
    (opt,), _ = m.configure_optimizers()
    assert torch.equal(m.student_model.P.master, w0)
    m.training_step(good, 0).backward()
    with torch.cuda.stream(m._stu_stream):
        torch.cuda._sleep(1_000_000_000)     # AdamW t queues behind this
    raised = []
    _attempt(opt.step, raised)
    opt.zero_grad()
    _attempt(lambda: m.training_step(bad, 1).backward(), raised)
    if not raised:
        _attempt(opt.step, raised)
    if not raised:
        _attempt(m.check_errors, raised)
    torch.cuda.synchronize()
    assert len(raised) == 1 and "image-token count" in raised[0], raised
    upd = (m.student_model.P.master - w0).double()
    assert float(upd.abs().max()) > 0, "step t's valid update was skipped"
    cos = float((upd @ ref_upd) / (upd.norm() * ref_upd.norm()))
    assert cos >= 0.999 and abs(float(upd.norm() / ref_upd.norm()) - 1) <= 1e-3, cos


def test_ce_only_accepts_minus100_and_rejects_out_of_vocab(dev):
    K = _K()
    meta, _ = load("bd")
    m = K.LlavaOnevisionModule("tiny-student")
    (opt) = m.configure_optimizers()
    b = batch(meta, dev)
    b["labels"] = b["labels"].clone()
    b["labels"][0, 3:9] = -100            # padding: ignored by the CE (DM:141)
    m.training_step(b, 0).backward()
    opt.step()
    b["labels"][0, 12] = 10 ** 7          # a target outside the vocabulary
    m.training_step(b, 1).backward()
    with pytest.raises(RuntimeError, match="out of bounds"):
        opt.step()
        m.check_errors()


@pytest.mark.parametrize("kind", ["lb", "fb"])
def test_loss_group_size_one_equals_accumulated_single_samples(kind, dev):
    """loss_group_size=1 on a 2-sample batch == the reference's bs=1 x accumulate 2:
    two single-sample micro-batches, each loss / 2, accumulated before one step."""
    K = _K()
    cls = K.LogitBasedKD if kind == "lb" else K.FeatureBasedKD
    meta, _ = load(kind)
    b = batch(meta, dev)
    grouped = cls("tiny-student", "tiny-teacher", loss_group_size=1)
    tot_g = grouped.training_step(b, 0)
    tot_g.backward()
    torch.cuda.synchronize()
    g_grouped = _grads(grouped)
    acc = cls("tiny-student", "tiny-teacher", accumulate_grad_batches=2)
    tots = []
    for i in range(2):
        bi = {k: (v[i:i + 1] if isinstance(v, torch.Tensor) else v) for k, v in b.items()}
        t = acc.training_step(bi, i)
        (t / 2).backward()
        tots.append(t.item())
    torch.cuda.synchronize()
    assert tot_g.item() == pytest.approx(sum(tots) / 2, rel=1e-4)
    _close_grads(g_grouped, _grads(acc))
    # and the coupled whole-batch loss differs (LoCa's overrides / NT-Xent's negatives span it)
    whole = cls("tiny-student", "tiny-teacher")
    assert whole.forward(b).item() != pytest.approx(tot_g.item(), rel=1e-7)


def test_checkpoint_reload_with_reference_keywords(dev, tmp_path):
    """evaluate_onevision.py:65-73 and BDT:86-91 call load_from_checkpoint with keywords
    (model names, processor, torch_dtype, map_location, phase)."""
    K = _K()
    m = K.OnlineKnowledgeDistillationLLavaOneVision("tiny-student", "tiny-teacher", phase=3)
    p = tmp_path / "dt3.ckpt"
    m.save_checkpoint(str(p))
    r = K.OnlineKnowledgeDistillationLLavaOneVision.load_from_checkpoint(
        str(p), model_name_student="tiny-student", model_name_teacher="tiny-teacher", processor=None,
        torch_dtype=torch.float16, map_location=torch.device("cpu"))
    assert r.phase == 3 and torch.equal(r.student_model.P.flat, m.student_model.P.flat)
    r1 = K.OnlineKnowledgeDistillationLLavaOneVision.load_from_checkpoint(str(p), phase=1)
    assert r1.phase == 1
    bd = K.LlavaOnevisionModule("tiny-student", seed_student=7)
    pb = tmp_path / "bd.ckpt"
    bd.save_checkpoint(str(pb))
    ck = torch.load(str(pb), weights_only=True)
    assert all(k.startswith("model.") for k in ck["state_dict"])      # the reference's self.model
    rb = K.LlavaOnevisionModule.load_from_checkpoint(str(pb), model_name="tiny-student", processor=None,
                                                     torch_dtype=torch.float16)
    assert torch.equal(rb.student_model.P.flat, bd.student_model.P.flat)
    # the knobs that change the objective / the update survive a reload without keywords
    lb = K.LogitBasedKD("tiny-student", "tiny-teacher", loss_group_size=1, accumulate_grad_batches=4)
    pl = tmp_path / "lb.ckpt"
    lb.save_checkpoint(str(pl))
    rl = K.LogitBasedKD.load_from_checkpoint(str(pl))
    assert rl.loss_group_size == 1 and rl.accumulate_grad_batches == 4 and rl.teacher_fp8 is False


_DP_CHILD = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, {repo!r}); sys.path.insert(0, {golden!r})
from model_fixtures import batch, load
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
meta, _ = load("lb")
b = batch(meta, torch.device("cuda:0"))
bi = {{k: (v[rank:rank + 1] if isinstance(v, torch.Tensor) else v) for k, v in b.items()}}
m = K.LogitBasedKD("tiny-student", "tiny-teacher", loss_group_size=1)
m._gsync.bucket_bytes = 1 << 16          # several buckets, launched during the backward
loss = m.training_step(bi, 0)
loss.backward()
lo, hi = m._trainable_range()
m._gsync.finish(lo, hi)
torch.cuda.synchronize()
torch.save({{"grad": m.student_model.P.grad[lo:hi].cpu(), "loss": loss.item()}}, {out!r} + f".{{rank}}")
dist.destroy_process_group()
'''


def test_two_rank_dp_step_equals_union_batch(dev, tmp_path):
    """Two ranks (fresh processes on the same GPU, gloo) with one sample each and
    loss_group_size=1 reduce to the same gradient as one process on both samples."""
    K = _K()
    meta, _ = load("lb")
    m = K.LogitBasedKD("tiny-student", "tiny-teacher", loss_group_size=1)
    tot = m.training_step(batch(meta, dev), 0)
    tot.backward()
    torch.cuda.synchronize()
    ref = _grads(m).float().cpu()
    out = str(tmp_path / "dp")
    script = tmp_path / "child.py"
    script.write_text(_DP_CHILD.format(repo=str(REPO), golden=str(REPO / "tests" / "golden"), out=out))
    port = 29700 + os.getpid() % 200
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env))
    for p in procs:
        assert p.wait(timeout=600) == 0
    res = [torch.load(out + f".{r}", weights_only=True) for r in range(2)]
    assert torch.equal(res[0]["grad"], res[1]["grad"])                 # replicas agree exactly
    assert tot.item() == pytest.approx((res[0]["loss"] + res[1]["loss"]) / 2, rel=1e-4)
    _close_grads(res[0]["grad"].double(), ref.double())


_RCCL_CHILD = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, {repo!r}); sys.path.insert(0, {golden!r})
from model_fixtures import batch, load
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
meta, _ = load("lb")
b = batch(meta, dev)


def run(m):
    (opt,), _ = m.configure_optimizers()
    w0 = m.student_model.P.master.clone()
    side = torch.cuda.Stream()               # a non-default caller stream, as bench.py's
    with torch.cuda.stream(side):
        for i in range(3):
            m.training_step(b, i).backward()
            opt.step()
            opt.zero_grad()
        m.training_step(b, 3).backward()     # grads read after backward: reduced (DDP)
        g = m.student_model.P.grad.clone()
    torch.cuda.synchronize()
    return (m.student_model.P.master - w0).double(), g.double()


def close(a, b):   # atomics in the embedding / bias gradients: not bit-exact run to run
    cos = float((a @ b) / (a.norm() * b.norm()))
    nr = float(a.norm() / b.norm())
    assert cos >= 0.9999 and abs(nr - 1) <= 2e-3, (cos, nr)


ref = run(K.LogitBasedKD("tiny-student", "tiny-teacher"))
dist.init_process_group("nccl", device_id=dev)
m = K.LogitBasedKD("tiny-student", "tiny-teacher", grad_comm_dtype={comm})
assert m._gsync is not None and m._gsync.avg_in_collective
m._gsync.bucket_bytes = 1 << 16          # several buckets, launched during the backward
got = run(m)
dist.barrier()
dist.destroy_process_group()
close(got[0], ref[0])   # the weight update of 3 RCCL-synced steps
close(got[1], ref[1])   # the 4th backward's gradient
print("rccl ok")
'''


@pytest.mark.parametrize("comm", ["None", "torch.bfloat16"])
def test_rccl_world1_steps_equal_local(comm, tmp_path):
    """The DP path on RCCL (backend "nccl": async bucketed AVG all-reduces launched on the
    student stream during the backward, awaited on the student stream before AdamW) on a
    one-rank group: three full steps give the same weight update and gradients as the module
    without a process group (the mean over one rank is the identity) — with fp32 buckets, and
    with bf16 buckets (grad_comm_dtype: the gradient rounded to bf16 on the way, the update
    within the same cosine / 2e-3 norm tolerance)."""
    script = tmp_path / "child.py"
    script.write_text(_RCCL_CHILD.format(repo=str(REPO), golden=str(REPO / "tests" / "golden"), comm=comm))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29900 + os.getpid() % 90))
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


class _RecordingDist:
    """A stand-in process group for GradSync (one rank, nothing on the wire): records where in
    the student backward each bucket is launched -- by kd_model_backward's per-part callbacks
    (include/kdstep.h ABI 9) or by GradSync.end after the backward."""

    class ReduceOp:
        AVG, SUM = "avg", "sum"

    class _Work:
        def wait(self):
            pass

    def __init__(self):
        self.launched = []

    def get_world_size(self):
        return 1

    def get_backend(self):
        return "nccl"

    def all_reduce(self, t, op=None, async_op=False):
        self.launched.append(int(t.numel()))
        return self._Work()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("phase", [3, 2])
def test_vit_gradient_buckets_launch_during_the_backward(phase, dev):
    """BASELINE c4 (DT phase 3, every student tower trainable) / c3 (phase 2, ViT frozen) at the real
    widths and full depth, bs 1: the data-parallel buckets are launched as kd_model_backward makes
    each part of the flat gradient final -- the Qwen2 layers, then embed_tokens / projector, then the
    SigLIP layers -- so what GradSync.end launches after the backward (grad_allreduce
    .bytes_after_backward in bench.py) is at most one 256 MB bucket plus the SigLIP patch / position
    embeddings (round 5 launched the whole ViT + projector + embed_tokens, 2.15 GB, there).
    Every trainable element is reduced exactly once."""
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.dp import GradSync
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    K = _K()
    m = K.OnlineKnowledgeDistillationLLavaOneVision("llava-hf/llava-onevision-qwen2-0.5b-ov-hf",
                                                    "llava-hf/llava-onevision-qwen2-7b-ov-hf", phase=phase)
    if phase == 2:
        m.freeze_student_vision_layers()
    rec = _RecordingDist()
    m._gsync = GradSync(rec, m.student_model.P.grad)
    loss = m.training_step(synthetic_batch(1, dev, L=1536, seed=0), 0)
    loss.backward()
    torch.cuda.synchronize()
    gs = m._gsync
    lo, hi = m._trainable_range()
    assert sum(gs.last_buckets) == hi - lo                          # the trainable range, once
    tail_bytes = gs.last_tail * 4
    emb = m.student_model.P.regions["vision"][0]
    vis_embed = min(off for n, (off, _) in m.student_model.P.offsets.items()
                    if ".encoder.layers.0." in n) - emb              # patch + position embeddings
    assert tail_bytes <= gs.bucket_bytes + 4 * vis_embed, tail_bytes
    assert tail_bytes <= 0.6e9
    assert len(gs.last_buckets) >= (8 if phase == 3 else 5), gs.last_buckets
