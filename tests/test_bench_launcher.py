"""bench.py --gpus N starts its own ranks (CPU, gloo, --dry: no model).

The driver's scaling command is `bench.py --gpus N`; without a torch.distributed launcher
bench.py must start N ranks itself (one process per GPU, torch.distributed.run as a child
process) and report n_gpus = N with every rank's time; under a launcher WORLD_SIZE must
equal N.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(REPO / "bench.py")] + args, cwd=REPO, env=env, capture_output=True,
                          text=True, timeout=timeout)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks():
    r = _run(["--gpus", "2", "--dry", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["dry"]
    assert len(d["per_rank_ms_per_step"]) == 2
    # value = steps of all ranks / the slowest rank's time
    slowest = max(d["per_rank_ms_per_step"]) * d["steps"] * 1e-3
    assert abs(d["value"] - 2 * d["steps"] / slowest) <= 0.02 * d["value"]


def test_single_rank_default():
    r = _run(["--dry", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _json_line(r.stdout)["n_gpus"] == 1


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry", "--steps", "1"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_parent_counts_gpus_without_starting_hip(tmp_path, monkeypatch):
    """The launcher parent counts devices from the KFD topology in sysfs, never through HIP: after
    the count torch.cuda is still uninitialised (so the parent holds no GPU context while its
    ranks run).  A fake topology: two GPU nodes (gfx_target_version != 0) and one CPU node."""
    import torch
    sys.path.insert(0, str(REPO))
    import bench
    for i, ver in enumerate(("0", "90500", "90500")):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 8\nsimd_count {0 if ver == '0' else 1024}\n"
                                      f"gfx_target_version {ver}\n")
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.visible_gpu_count(str(tmp_path)) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.visible_gpu_count(str(tmp_path)) == 1
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    assert bench.visible_gpu_count(str(tmp_path / "missing")) is None
    bench.visible_gpu_count()          # the real sysfs (whatever this host has)
    assert not torch.cuda.is_initialized()


def _allreduce_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(REPO))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _GS:
        last_buckets = [1 << 16, 1 << 15, 1000]
        last_tail = 1000
        comm_dtype = None

    class _M:
        _gsync = _GS()
    try:
        q.put((rank, bench.allreduce_cost(_M(), dist, "cpu", world)))
    finally:
        dist.destroy_process_group()


def test_allreduce_cost_schema_gloo():
    """bench.py's grad_allreduce object (the N > 1 line's DP exchange), model-free on 2 gloo ranks:
    bucket count, bytes (fp32), dtype, the standalone time (max over ranks: every rank reports the
    same) and the ring bus bandwidth 2 (N - 1) / N x bytes / time."""
    import multiprocessing as mp
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_allreduce_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = res[0], res[1]
    n = (1 << 16) + (1 << 15) + 1000
    for r in (a, b):
        assert set(r) == {"buckets", "bytes", "dtype", "bytes_after_backward", "standalone_ms", "ring_bus_GBps",
                          "measured"}
        assert r["bytes_after_backward"] == 4000
        assert r["buckets"] == 3 and r["bytes"] == 4 * n and r["dtype"] == "float32"
        assert r["standalone_ms"] > 0
        bw = 2 * (2 - 1) / 2 * r["bytes"] / (r["standalone_ms"] * 1e-3) / 1e9
        assert abs(r["ring_bus_GBps"] - round(bw, 1)) <= 0.11
    assert a["standalone_ms"] == b["standalone_ms"]
