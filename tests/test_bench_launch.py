"""bench.py's launcher contract (CPU, gloo): `python bench.py --gpus N` with no WORLD_SIZE in the
environment starts N ranks itself (torch.distributed.run as a child process, before any GPU call),
and a launcher whose WORLD_SIZE disagrees with --gpus is refused.  --launch-check stops each rank
right after the control-plane rendezvous, so no GPU is needed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_n_without_launcher_starts_n_ranks():
    for n in (2, 3):
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                             env=_env(), capture_output=True, text=True, timeout=240)
        assert out.returncode == 0, out.stderr[-2000:]
        lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, out.stdout   # one JSON line, from rank 0 only
        rec = json.loads(lines[0])
        assert rec["world"] == n
        assert sorted(r["rank"] for r in rec["ranks"]) == list(range(n))
        assert sorted(r["local_rank"] for r in rec["ranks"]) == list(range(n))
        assert len({r["pid"] for r in rec["ranks"]}) == n   # one process per rank


def test_world_size_must_match_gpus():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--launch-check"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stdout + out.stderr


def test_single_gpu_default_does_not_launch():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launch-check"],
                         env=_env(), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["world"] == 1 and rec["ranks"][0]["rank"] == 0
