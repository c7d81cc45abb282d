"""bench.py's multi-GPU launch contract on CPU: `--gpus N` without a torch.distributed environment
starts N ranks itself (torch.distributed.run children; the parent never touches the GPU), and a rank
whose WORLD_SIZE disagrees with --gpus refuses to report."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True, timeout=240,
                          env=env, cwd=REPO)


def test_gpus_2_forms_two_ranks():
    p = _run(["--gpus", "2", "--dist-backend", "gloo", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout   # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_formed"] == 2 and d["world_size"] == 2


def test_gpus_3_forms_three_ranks():
    p = _run(["--gpus", "3", "--dist-backend", "gloo", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 3 and d["ranks_formed"] == 3


def test_world_size_mismatch_is_an_error():
    p = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=1" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
