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
