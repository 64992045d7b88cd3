"""CPU (gloo) tests of the query-row sharding collectives: partitioning and the fixed-chunk
all-gather of ragged row slabs (RowExchange) through its persistent buffers, checked against a
test-side restatement of the HIP reassembly.  world_size 2, 3 and 8 (the C5 node split) processes on 127.0.0.1."""
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


def _assemble_host(recv, world, B, C, H, W):
    """Test-side restatement of ecorr_rows_assemble (include/ecorr.h): chunk r starts with rank
    r's rows as [B][C][rows_r][W]."""
    from eraft_amd.rowshard import row_partition
    starts, counts = row_partition(H, world)
    chunks = recv.view(world, -1)
    out = torch.empty((B, C, H, W), dtype=recv.dtype)
    for r in range(world):
        n = B * C * counts[r] * W
        out[:, :, starts[r]:starts[r] + counts[r]] = chunks[r, :n].view(B, C, counts[r], W)
    return out


def _worker(rank, world, port, H, W, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from eraft_amd.rowshard import RowExchange, row_partition
        starts, counts = row_partition(H, world)
        B, C = 3, 5
        full = torch.arange(B * C * H * W, dtype=torch.float32).reshape(B, C, H, W)
        ex = RowExchange(H)
        ok = True
        for it in range(2):   # the persistent buffers are reused across calls
            slab = ex.send_slab(B, C, W)
            assert tuple(slab.shape) == (B, C, counts[rank], W)
            slab.copy_(full[:, :, starts[rank]:starts[rank] + counts[rank]] + it)
            recv = ex.gather_chunks(B, C, W)
            assert recv.numel() == world * B * C * max(counts) * W
            ok = ok and bool(torch.equal(_assemble_host(recv, world, B, C, H, W), full + it))
        q.put((rank, ok, counts))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - report to the parent
        q.put((rank, repr(e), None))


@pytest.mark.parametrize("world,H", [(2, 60), (3, 92), (2, 7), (8, 92)])   # 8: the C5 split over a node
def test_row_exchange_chunks_reassemble(world, H):
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


def test_gather_rows_refuses_other_partitions():
    from eraft_amd.rowshard import gather_rows
    if not dist.is_initialized():
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with pytest.raises(ValueError):
            gather_rows(torch.zeros(1, 1, 3, 4), [3, 1])       # not world 1's partition of 4 rows
        with pytest.raises(RuntimeError):
            from eraft_amd.rowshard import RowShardedCorrBlock
            RowShardedCorrBlock(torch.zeros(1, 4, 3, 4), torch.zeros(1, 4, 3, 4))   # CPU: no HIP path
    finally:
        dist.destroy_process_group()
