"""Query-row sharded CorrBlock on the GPU: 2 ranks on cuda:0 (gloo carries CUDA tensors), each
building only its query rows from row slabs (fmap2 all-gathered), must reproduce the unsharded
CorrBlock bit for bit -- the per-element MFMA k order does not depend on the tiling -- and the
gathered lookup must equal the unsharded lookup exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import eraft_amd
        import prng
        from eraft_amd.rowshard import RowShardedCorrBlock, row_partition
        B, D, H, W = 2, 256, 23, 40            # ragged rows: 12 + 11
        f1 = torch.from_numpy(prng.normal(71, (B, D, H, W))).cuda()
        f2 = torch.from_numpy(prng.normal(72, (B, D, H, W))).cuda()
        coords = torch.from_numpy(prng.coords_with_flow(73, B, H, W, 4.0)).cuda()
        starts, counts = row_partition(H, world)
        r0, rr = starts[rank], counts[rank]
        with torch.no_grad():
            full = eraft_amd.CorrBlock(f1, f2)
            ref = full(coords)
            sh = RowShardedCorrBlock.from_row_slabs(f1[:, :, r0:r0 + rr], f2[:, :, r0:r0 + rr], H)
            out = sh(coords)
            rep = RowShardedCorrBlock(f1, f2)   # replicated-fmap constructor
            out2 = rep(coords)
        torch.cuda.synchronize()
        rows = slice(B * 0, None)
        lvl_ok = all(
            torch.equal(sh.corr_pyramid[i].view(B, rr * W, -1),
                        full.corr_pyramid[i].view(B, H * W, -1)[:, r0 * W:(r0 + rr) * W])
            for i in range(4))
        q.put((rank, lvl_ok, bool(torch.equal(out, ref)), bool(torch.equal(out2, ref)), None))
        del rows
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, False, False, False, repr(e)))


def test_rowshard_two_ranks_bit_exact():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, lvl_ok, out_ok, out2_ok, err in res:
        assert err is None, err
        assert lvl_ok, f"rank {rank}: pyramid slab differs from the unsharded pyramid"
        assert out_ok and out2_ok, f"rank {rank}: gathered lookup differs"
    assert np.all([r[2] for r in res])
