"""bench.py's rank launcher (the command the driver's scaling run uses: `python bench.py --gpus N`
with no launcher around it).  CPU: `--dry-launch` starts the ranks, joins the gloo control plane
and stops before any GPU work.  GPU: on a 1-GPU box `--gpus 2` must fail loudly, never print a
one-rank line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env=None, timeout=180):
    return subprocess.run([sys.executable, BENCH] + args, env=env or _env(), capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("n,workload", [(2, "c3"), (3, "c4"), (2, "c5")])
def test_gpus_n_starts_n_ranks(n, workload):
    p = _run(["--gpus", str(n), "--dry-launch", "--workload", workload])
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout                   # rank 0's line only
    d = json.loads(lines[0])
    assert d["dry_launch"] and d["world_size"] == n and d["gpus"] == n and d["workload"] == workload
    assert d["launcher"] == "bench.py"
    assert [r["rank"] for r in d["ranks"]] == list(range(n))
    assert [r["local_rank"] for r in d["ranks"]] == list(range(n))
    assert len({r["pid"] for r in d["ranks"]}) == n    # n distinct processes


def test_one_gpu_needs_no_launch():
    p = _run(["--dry-launch"])
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout.strip())
    assert d["world_size"] == 1 and d["launcher"] == "none"


def test_world_size_disagreeing_with_gpus_is_refused():
    p = _run(["--gpus", "2", "--dry-launch"], env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "disagree" in p.stderr
    assert not p.stdout.strip()


def test_too_few_gpus_fails_every_rank_without_a_line():
    # this container has no GPU: two ranks must both refuse (exit 3) and the launch fail
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"])
    assert p.returncode != 0
    assert "GPU(s)" in p.stderr
    assert not p.stdout.strip()


@pytest.mark.gpu
def test_gpus_2_on_a_one_gpu_box_fails_loudly():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("node has >= 2 GPUs")
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"], timeout=120)
    assert p.returncode != 0
    assert "one rank per GPU is required" in p.stderr
    assert not p.stdout.strip()
