"""World-size-2 run of the batch-sharded bench path (BASELINE configs[3]).

bench.py launched by torch.distributed.run with 2 processes, both on cuda:0 (BENCH_SINGLE_DEVICE=1:
gloo for the timing max-reduce, set in the launcher's environment before any GPU call): each rank
builds and looks up its OWN batch of pairs (seed 1234 + rank), no data-path collective, and rank 0
reports the whole job.  Checks: n_gpus, the global batch (2 x 16), distinct per-rank inputs, and
value = pairs of all ranks / the max-reduced elapsed time.  One GPU shared by two ranks measures
the path, not the scaling: the 1/2/4/8-GPU curve is the driver's 8-GPU run.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpu_untouched():
    # Precondition: this process has not initialised the GPU.  The launcher is a forked child of
    # the pytest process; a child that execs from a GPU-initialised parent can take the machine
    # down on this pool.  conftest.py orders these tests first in the session; if a reordering ever
    # runs a GPU test before them, fail here instead of spawning the ranks.
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        pytest.fail("the spawning tests must run before any test initialises the GPU in this "
                    "process (conftest.py puts them first); run alone: pytest tests/test_batch_shard_gpu.py")


@pytest.mark.parametrize("launcher", ["bench_itself", "torchrun"])
def test_two_rank_batch_shard(launcher):
    """`bench_itself`: `python bench.py --gpus 2` with no launcher around it -- the form a driver
    may run for its 1/2/4/8 curve -- must start the 2 ranks itself."""
    _gpu_untouched()
    steps, B = 2, 16
    env = dict(os.environ, BENCH_SINGLE_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", "1",
             "--batch", str(B), "--no-next", "--no-cpu-baseline"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + bench
    else:
        cmd = [sys.executable] + bench
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 alone prints
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == steps and res["scaling"] == "weak"
    cfg = res["config"]
    assert cfg["global_batch"] == 2 * B
    assert cfg["rank_seeds"] == [1234, 1235]
    c0, c1 = cfg["rank_input_checksums"]
    assert c0 != c1, "both ranks built the same pairs"
    elapsed = res["ms_per_step"] * steps / 1e3
    assert res["value"] == pytest.approx(2 * B * steps / elapsed, rel=1e-3)
    assert res["kernels"]["build"]["ms_per_launch"] > 0 and res["kernels"]["lookup"]["ms_per_launch"] > 0


def test_two_rank_rowshard_bench():
    """BASELINE configs[4] through bench.py itself: `bench.py --mode rowshard --gpus 2` with no launcher
    starts 2 ranks (both on cuda:0 over gloo here), shards the 92 query rows 46 / 46, and checks one
    sharded lookup against the unsharded CorrBlock after the timed region (bit-exact)."""
    _gpu_untouched()
    env = dict(os.environ, BENCH_SINGLE_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mode", "rowshard", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--no-next", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["scaling"] == "strong"
    assert res["config"]["row_partition"] == [46, 46]
    assert res["config"]["check_vs_unsharded"] == "bit-exact"
