"""bench.py's --gpus contract, the part that runs without a GPU: a launcher whose WORLD_SIZE differs
from --gpus N is refused before any device call; the N-rank self-launch itself
is exercised on the GPU box (tests/test_batch_shard_gpu.py, launcher=bench_itself)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=120)


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_zero_gpus_refused():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus 0" in r.stderr
