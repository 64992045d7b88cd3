"""CPU (gloo) tests of the query-row sharding collectives: partitioning and the padded
all-gather that reassembles ragged row slabs.  world_size 2 and 3 processes on 127.0.0.1."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (puts the repo root on sys.path)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, H, W, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from eraft_amd.rowshard import gather_rows, row_partition
        starts, counts = row_partition(H, world)
        full = torch.arange(3 * 5 * H * W, dtype=torch.float32).reshape(3, 5, H, W)
        slab = full[:, :, starts[rank]:starts[rank] + counts[rank]].contiguous()
        got = gather_rows(slab, counts)
        q.put((rank, bool(torch.equal(got, full)), counts))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - report to the parent
        q.put((rank, repr(e), None))


@pytest.mark.parametrize("world,H", [(2, 60), (3, 92), (2, 7)])
def test_gather_rows_reassembles(world, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, 9, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, counts in res:
        assert ok is True, (rank, ok)
        assert sum(counts) == H and max(counts) - min(counts) <= 1


def test_row_partition_matches_survey_split():
    from eraft_amd.rowshard import row_partition
    starts, counts = row_partition(92, 8)          # 12,12,12,12,11,11,11,11
    assert counts == [12, 12, 12, 12, 11, 11, 11, 11]
    assert starts == [0, 12, 24, 36, 48, 59, 70, 81]
    with pytest.raises(ValueError):
        row_partition(3, 4)
