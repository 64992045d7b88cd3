"""Query-row sharded CorrBlock on the GPU: 2 ranks on cuda:0 (gloo carries CUDA tensors), each
building only its query rows, must reproduce the unsharded CorrBlock bit for bit -- the
per-element MFMA k order does not depend on the tiling -- and the gathered lookup (plain 324
channels, and fused relu(convc1(lookup)) 256 channels) must equal the unsharded one exactly.
Cases: a ragged 23 x 40 map (12 + 11 rows) and BASELINE configs[4]'s shape, 1280 x 720 frames
= 92 x 160 fmaps, D = 256, B = 4.  The collective here is gloo (one GPU); the RCCL branch
(all_gather_into_tensor) runs only on multi-GPU nodes."""
import os
import socket

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


def _worker(rank, world, port, shape, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import eraft_amd
        import prng
        from eraft_amd.rowshard import RowShardedCorrBlock, row_partition
        B, D, H, W = shape
        f1 = torch.from_numpy(prng.normal(71, (B, D, H, W))).cuda()
        f2 = torch.from_numpy(prng.normal(72, (B, D, H, W))).cuda()
        coords = torch.from_numpy(prng.coords_with_flow(73, B, H, W, 4.0)).cuda()
        wt = torch.from_numpy(prng.normal(74, (256, 324, 1, 1), 0.05)).cuda()
        bias = torch.from_numpy(prng.normal(75, (256,), 0.1)).cuda()
        starts, counts = row_partition(H, world)
        r0, rr = starts[rank], counts[rank]
        res = {}
        with torch.no_grad():
            full = eraft_amd.CorrBlock(f1, f2)
            ref = full(coords)
            ref_fused = {m: full.lookup_conv1x1_relu(coords, wt, bias, mode=m) for m in ("fused", "split")}
            sh = RowShardedCorrBlock.from_row_slabs(f1[:, :, r0:r0 + rr], f2[:, :, r0:r0 + rr], H)
            for it in range(2):   # persistent exchange buffers, reused
                res[f"plain{it}"] = bool(torch.equal(sh(coords), ref))
                for m in ("fused", "split"):   # both convc1 modes: bitwise the unsharded rows
                    res[f"{m}{it}"] = bool(torch.equal(sh.lookup_conv1x1_relu(coords, wt, bias, mode=m), ref_fused[m]))
            res["local"] = bool(torch.equal(sh.lookup_local(coords[:, :, r0:r0 + rr].contiguous()),
                                            ref[:, :, r0:r0 + rr]))
            rep = RowShardedCorrBlock(f1, f2)   # replicated-fmap constructor
            res["replicated"] = bool(torch.equal(rep(coords), ref))
            torch.cuda.synchronize()
            res["pyramid"] = all(
                torch.equal(sh.corr_pyramid[i].view(B, rr * W, -1),
                            full.corr_pyramid[i].view(B, H * W, -1)[:, r0 * W:(r0 + rr) * W])
                for i in range(4))
            # the loud contract: mismatched fmaps, coords on the wrong device / shape
            neg = []
            for bad in (lambda: RowShardedCorrBlock(f1, f2[:, :, :-1].contiguous()),
                        lambda: RowShardedCorrBlock(f1, f2.cpu()),
                        lambda: sh.lookup_local(coords[:, :, r0:r0 + rr].cpu()),
                        lambda: sh.lookup_local(coords[:, :, :1].contiguous()),
                        lambda: sh.lookup_conv1x1_relu(coords, wt.cpu(), bias),
                        lambda: sh.lookup_conv1x1_relu(coords, wt[:, :100].contiguous(), bias),
                        lambda: full.lookup_conv1x1_relu(coords, wt, bias.cpu())):
                try:
                    bad()
                    neg.append(False)
                except (RuntimeError, TypeError):
                    neg.append(True)
            res["negative"] = all(neg)
        q.put((rank, res, None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, {}, repr(e)))


@pytest.mark.parametrize("shape", [(2, 256, 23, 40), (4, 256, 92, 160)], ids=["23x40_ragged", "c5_92x160_b4"])
def test_rowshard_two_ranks_bit_exact(shape):
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, shape, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, r, err in res:
        assert err is None, err
        bad = [k for k, v in r.items() if not v]
        assert not bad, f"rank {rank}: {bad}"
    assert all(len(r[1]) == 10 for r in res)   # plain, fused, split x 2 iterations + 4 checks


def _rccl_worker(port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        import prng
        from eraft_amd.rowshard import RowExchange
        B, C, H, W = 2, 324, 23, 40
        full = torch.from_numpy(prng.normal(81, (B, C, H, W))).cuda()
        ex = RowExchange(H)
        ok = []
        for it in range(2):   # persistent buffers
            ex.send_slab(B, C, W, device=full.device).copy_(full + it)
            ok.append(bool(torch.equal(ex.gather(B, C, W, full.device), full + it)))
        q.put((all(ok), dist.get_backend(), None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((False, None, repr(e)))


def test_row_exchange_over_rccl_one_rank():
    """The RCCL branch of the exchange (all_gather_into_tensor into the persistent receive buffer,
    then ecorr_rows_assemble) on the one GPU this box has: a 1-rank "nccl" group.  Multi-rank RCCL
    runs only on multi-GPU nodes (the driver's scaling bench)."""
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    ok, backend, err = q.get(timeout=180)
    p.join(timeout=60)
    assert err is None, err
    assert backend == "nccl" and ok


@pytest.mark.parametrize("world,B,C,H,W", [(3, 2, 5, 7, 9), (8, 4, 324, 92, 160), (2, 1, 3, 5, 8), (4, 2, 7, 4, 13)])
def test_rows_assemble_kernel(world, B, C, H, W):
    """ecorr_rows_assemble alone on chunk data of the all-gather layout (16-byte and scalar paths,
    ragged partitions), against a test-side reassembly."""
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible")
    import eraft_amd
    from eraft_amd import _lib
    from eraft_amd.rowshard import row_partition
    starts, counts = row_partition(H, world)
    chunk = B * C * max(counts) * W
    recv = torch.randn(world * chunk, device="cuda")
    out = torch.full((B, C, H, W), float("nan"), device="cuda")
    eraft_amd.lib()
    _lib.check(_lib.lib().ecorr_rows_assemble(recv.data_ptr(), chunk, world, B, C, H, W, out.data_ptr(),
                                              _lib.stream_of(out)), "rows assemble")
    ref = torch.empty_like(out)
    ch = recv.view(world, chunk)
    for r in range(world):
        ref[:, :, starts[r]:starts[r] + counts[r]] = ch[r, :B * C * counts[r] * W].view(B, C, counts[r], W)
    assert torch.equal(out, ref)
    # loud on a chunk too small for the partition
    assert _lib.lib().ecorr_rows_assemble(recv.data_ptr(), chunk - 1, world, B, C, H, W, out.data_ptr(),
                                          _lib.stream_of(out)) != 0
