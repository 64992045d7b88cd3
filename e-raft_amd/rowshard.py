"""Query-row sharded CorrBlock for high-resolution frames (BASELINE configs[4]).

The all-pairs volume row of query pixel p depends only on fmap1[:, :, p] and ALL of fmap2, and
the pyramid pools over fmap2's (target) dims.  So the query pixels split cleanly by image rows:
rank r owns rows [start_r, start_r + rows_r) of the 1/8-resolution map, builds the pyramid for
those queries only (1/world of the GEMM and of the 1.15 GB/pair volume at 1280x720), and answers
lookups for them with no communication.  The exchanges are:

  1. fmap2 all-gather, once per frame pair, when the feature maps arrive as row slabs (a
     spatially sharded fnet): RowShardedCorrBlock.from_row_slabs;
  2. per GRU iteration, the all-gather of the lookup output -- ERAFT.forward keeps the GRU
     replicated and needs the full map on every rank (eraft.py:128-132).  __call__ gathers the
     324-channel lookup; lookup_conv1x1_relu gathers the 256-channel relu(convc1(lookup)) that
     BasicMotionEncoder computes from it (update.py:67,74), 21% fewer bytes.

Every exchange is one all-gather of fixed-size chunks (RowExchange): the local result is written
straight into a persistent send chunk ([B][C][rows_r][W] at its start, padding behind), the
collective lands in a persistent receive buffer [world][chunk], and one HIP kernel
(ecorr_rows_assemble) writes the [B][C][H][W] map from it.  No padding copy, no torch.cat.  The
collective is RCCL over xGMI with the "nccl" backend (all_gather_into_tensor); any other backend
(the CPU tests use gloo) gets all_gather into views of the same receive buffer.
"""
import os

import torch
import torch.distributed as dist

from . import _lib
from .corr import _no_grad_inputs, _require_device_f32
from .layout import formats, untile


def row_partition(H, world):
    """Contiguous near-equal row blocks: (starts, counts), counts differ by at most one (the
    first H % world ranks own one row more -- the partition ecorr_rows_assemble assumes)."""
    if world < 1 or H < world:
        raise ValueError(f"cannot split {H} rows over {world} ranks")
    base, extra = divmod(H, world)
    counts = [base + (1 if r < extra else 0) for r in range(world)]
    starts = [sum(counts[:r]) for r in range(world)]
    return starts, counts


class RowExchange:
    """All-gather of per-rank row slabs [B, C, rows_r, W] into the full [B, C, H, W].

    Buffers persist per (B, C, W, dtype, device): send = one chunk of B*C*max(rows)*W elements,
    recv = world chunks.  Usage: fill send_slab(...) in place, then gather(...).  gather_chunks
    (the collective alone) also runs on CPU tensors, which is how the gloo tests check the chunk
    layout; the reassembly is the HIP kernel and needs a HIP device.

    The send / receive buffers are reused by every gather, which is safe because the collective
    is synchronous and runs on the launch stream (NCCL/RCCL enqueue on the current stream): the
    next fill of the send chunk is stream-ordered after the previous collective read it.  Do not
    call gather_chunks with async_op or from a side stream, and do not hold a returned receive
    buffer across the next gather.
    """

    def __init__(self, H, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.H = H
        self.starts, self.counts = row_partition(H, self.world)
        self._bufs = {}

    def chunk_elems(self, B, C, W):
        return B * C * max(self.counts) * W

    def _buffers(self, B, C, W, dtype, device):
        key = (B, C, W, dtype, device)
        if key not in self._bufs:
            n = self.chunk_elems(B, C, W)
            self._bufs[key] = (torch.empty(n, dtype=dtype, device=device),
                               torch.empty(self.world * n, dtype=dtype, device=device))
        return self._bufs[key]

    def send_slab(self, B, C, W, dtype=torch.float32, device=None):
        """This rank's [B, C, rows_r, W] slab: a view of the start of the persistent send chunk."""
        send, _ = self._buffers(B, C, W, dtype, device)
        rr = self.counts[self.rank]
        return send[:B * C * rr * W].view(B, C, rr, W)

    def gather_chunks(self, B, C, W, dtype=torch.float32, device=None):
        """The collective: every rank's send chunk -> recv [world * chunk] (returned)."""
        send, recv = self._buffers(B, C, W, dtype, device)
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(recv, send, group=self.group)
        else:
            dist.all_gather(list(recv.view(self.world, -1).unbind(0)), send, group=self.group)
        return recv

    def gather(self, B, C, W, device):
        """Collective + reassembly of the float32 slabs filled through send_slab: [B, C, H, W]."""
        recv = self.gather_chunks(B, C, W, torch.float32, device)
        _require_device_f32("rows exchange buffer", recv)
        out = torch.empty((B, C, self.H, W), dtype=torch.float32, device=recv.device)
        with _lib.on_device(recv.device):
            _lib.check(_lib.lib().ecorr_rows_assemble(
                recv.data_ptr(), self.chunk_elems(B, C, W), self.world, B, C, self.H, W, out.data_ptr(),
                _lib.stream_of(out)), "RowExchange assemble")
        return out


def gather_rows(slab, counts, group=None):
    """All-gather per-rank row slabs [B, C, rows_r, W] (HIP float32) into the full
    [B, C, sum(rows), W] -- a one-off exchange (exchange 1); RowShardedCorrBlock keeps a
    RowExchange for the per-iteration one."""
    world = dist.get_world_size(group)
    H = sum(counts)
    if list(counts) != row_partition(H, world)[1]:
        raise ValueError(f"row counts {list(counts)} are not the contiguous near-equal partition of {H} rows")
    if world == 1:
        return slab.contiguous()
    _require_device_f32("slab", slab)
    B, C, rr, W = slab.shape
    ex = RowExchange(H, group)
    if rr != ex.counts[ex.rank]:
        raise RuntimeError(f"rank {ex.rank}: slab has {rr} rows, the partition gives it {ex.counts[ex.rank]}")
    ex.send_slab(B, C, W, device=slab.device).copy_(slab)
    return ex.gather(B, C, W, slab.device)


class RowShardedCorrBlock:
    """CorrBlock over a process group, queries sharded by image rows.

    RowShardedCorrBlock(fmap1, fmap2, ...)            full fmaps on every rank (replicated fnet);
    RowShardedCorrBlock.from_row_slabs(f1_rows, f2_rows, H, ...)   row slabs, fmap2 all-gathered.
    __call__(coords) takes the full [B, 2, H, W] coords (replicated GRU) and returns the full
    [B, C, H, W] lookup on every rank, bit-identical to the unsharded CorrBlock;
    lookup_conv1x1_relu(coords, weight, bias) returns the full relu(convc1(lookup)) the same way.
    """

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, group=None):
        _require_device_f32("fmap1", fmap1)
        _require_device_f32("fmap2", fmap2)
        _no_grad_inputs(fmap1, fmap2)
        if fmap1.dim() != 4 or fmap1.shape != fmap2.shape:
            raise RuntimeError(f"fmap shapes {tuple(fmap1.shape)} / {tuple(fmap2.shape)} differ "
                               "or are not [B, D, H, W]")
        if fmap1.device != fmap2.device:
            raise RuntimeError("fmap1 and fmap2 are on different devices")
        self._ex = RowExchange(fmap1.shape[2], group)
        self.group, self.rank, self.world = group, self._ex.rank, self._ex.world
        self.starts, self.counts = self._ex.starts, self._ex.counts
        r0, rr = self.starts[self.rank], self.counts[self.rank]
        self._init_local(fmap1[:, :, r0:r0 + rr].contiguous(), fmap2.contiguous(), num_levels, radius)

    @classmethod
    def from_row_slabs(cls, fmap1_rows, fmap2_rows, H, num_levels=4, radius=4, group=None):
        self = cls.__new__(cls)
        _require_device_f32("fmap1_rows", fmap1_rows)
        _require_device_f32("fmap2_rows", fmap2_rows)
        _no_grad_inputs(fmap1_rows, fmap2_rows)
        self._ex = RowExchange(H, group)
        self.group, self.rank, self.world = group, self._ex.rank, self._ex.world
        self.starts, self.counts = self._ex.starts, self._ex.counts
        if (fmap1_rows.dim() != 4 or fmap1_rows.shape[2] != self.counts[self.rank]
                or fmap2_rows.shape != fmap1_rows.shape):
            raise RuntimeError(f"rank {self.rank}: row slabs {tuple(fmap1_rows.shape)} / "
                               f"{tuple(fmap2_rows.shape)} do not match {self.counts[self.rank]} rows")
        if fmap1_rows.device != fmap2_rows.device:
            raise RuntimeError("fmap1_rows and fmap2_rows are on different devices")
        B, D, _, W = fmap2_rows.shape
        if self.world == 1:
            fmap2 = fmap2_rows.contiguous()
        else:                                                                # exchange 1
            self._ex.send_slab(B, D, W, device=fmap2_rows.device).copy_(fmap2_rows)
            fmap2 = self._ex.gather(B, D, W, fmap2_rows.device)
            self._ex._bufs.clear()   # one-off: do not keep the D-channel buffers
        self._init_local(fmap1_rows.contiguous(), fmap2, num_levels, radius)
        return self

    def _init_local(self, fmap1_rows, fmap2, num_levels, radius):
        self.num_levels, self.radius = num_levels, radius
        self._wcache = {}   # packed convc1 weights of this block (_lib.packed_conv1x1_weight)
        B, D, H, W = fmap2.shape
        self._shape = (B, D, H, W)
        self._device = fmap2.device
        self.q_count = self.counts[self.rank] * W
        self._h, self._w, self._off = _lib.layout(B * self.q_count, H, W, num_levels)
        with _lib.on_device(self._device):
            self._pyramid = _lib.build_pyramid(fmap1_rows, fmap2, B, D, H, W, self.q_count, num_levels,
                                               self._off, "RowShardedCorrBlock build")
        self._levels_cache = None

    @property
    def corr_pyramid(self):
        """This rank's levels in the reference layout [B*rows_r*W, 1, h_i, w_i] (a copy)."""
        if self._levels_cache is None:
            rows = self._shape[0] * self.q_count
            ntx = formats(self._shape[2], self._shape[3], self.num_levels)
            self._levels_cache = [
                untile(self._pyramid[self._off[i]:self._off[i + 1]], rows, self._h[i], self._w[i], ntx[i], i)
                for i in range(self.num_levels)]
        return self._levels_cache

    def _local_coords(self, coords_rows):
        B, _, H, W = self._shape
        rr = self.counts[self.rank]
        _require_device_f32("coords", coords_rows)
        _no_grad_inputs(coords_rows)
        if tuple(coords_rows.shape) != (B, 2, rr, W):
            raise RuntimeError(f"coords rows {tuple(coords_rows.shape)} != {(B, 2, rr, W)}")
        if coords_rows.device != self._device:
            raise RuntimeError("coords is on a different device than the pyramid")
        return coords_rows.contiguous()

    def _lookup_into(self, coords_rows, out):
        B, _, H, W = self._shape
        with _lib.on_device(self._device):
            _lib.check(_lib.lib().ecorr_lookup(
                self._pyramid.data_ptr(), coords_rows.data_ptr(), B, H, W, self.q_count,
                self.num_levels, self.radius, out.data_ptr(), _lib.stream_of(out)),
                "RowShardedCorrBlock lookup")
        return out

    def lookup_local(self, coords_rows):
        """Lookup for this rank's query rows: coords [B, 2, rows_r, W] -> [B, C, rows_r, W]."""
        coords_rows = self._local_coords(coords_rows)
        B, _, H, W = self._shape
        K = 2 * self.radius + 1
        C = self.num_levels * K * K
        out = torch.empty((B, C, self.counts[self.rank], W), dtype=torch.float32, device=self._device)
        return self._lookup_into(coords_rows, out)

    def _full_coords_rows(self, coords):
        B, _, H, W = self._shape
        if tuple(coords.shape) != (B, 2, H, W):
            raise RuntimeError(f"coords shape {tuple(coords.shape)} != {(B, 2, H, W)}")
        r0, rr = self.starts[self.rank], self.counts[self.rank]
        return self._local_coords(coords if rr == H else coords[:, :, r0:r0 + rr])

    def __call__(self, coords):
        B, _, H, W = self._shape
        coords_rows = self._full_coords_rows(coords)
        K = 2 * self.radius + 1
        C = self.num_levels * K * K
        if self.world == 1:
            out = torch.empty((B, C, H, W), dtype=torch.float32, device=self._device)
            return self._lookup_into(coords_rows, out)
        self._lookup_into(coords_rows, self._ex.send_slab(B, C, W, device=self._device))
        return self._ex.gather(B, C, W, self._device)                        # exchange 2

    def lookup_conv1x1_relu(self, coords, weight, bias=None, mode=None):
        """F.relu(conv1x1(self(coords), weight, bias)) for the full map on every rank: this rank's
        rows through the lookup + convc1 + ReLU (CorrBlock.lookup_conv1x1_relu, same `mode`), then
        the O-channel all-gather (exchange 2, fused form)."""
        mode = mode or os.environ.get("ECORR_CONVC1", "split")
        if mode not in ("split", "fused"):
            raise ValueError(f"mode {mode!r}: expected 'split' or 'fused'")
        B, _, H, W = self._shape
        coords_rows = self._full_coords_rows(coords)
        _require_device_f32("weight", weight)
        _no_grad_inputs(weight, *(() if bias is None else (bias,)))
        if weight.device != self._device or (bias is not None and bias.device != self._device):
            raise RuntimeError("weight / bias are on a different device than the pyramid")
        K = 2 * self.radius + 1
        C = self.num_levels * K * K
        O = weight.shape[0]
        if weight.numel() != O * C:
            raise RuntimeError(f"weight {tuple(weight.shape)} does not map {C} correlation channels")
        if bias is not None:
            _require_device_f32("bias", bias)
            if bias.numel() != O:
                raise RuntimeError(f"bias has {bias.numel()} elements, expected {O}")
            bias = bias.contiguous()
        if mode == "fused" and (O <= 0 or O % 64 != 0):
            raise RuntimeError(f"{O} output channels: the fused kernel needs a positive multiple of 64")
        if self.world == 1:
            out = torch.empty((B, O, H, W), dtype=torch.float32, device=self._device)
        else:
            out = self._ex.send_slab(B, O, W, device=self._device)
        with _lib.on_device(self._device):
            if mode == "split":
                wt = _lib.packed_conv1x1_weight(weight, O, C, "split", _lib.stream_of(out), self._wcache)
                G = 3 * self.num_levels
                corr = torch.empty((B, C, self.q_count), dtype=torch.float32, device=self._device)
                qmax = torch.empty((B, G, self.q_count), dtype=torch.float32, device=self._device)
                _lib.check(_lib.lib().ecorr_lookup_qmax(
                    self._pyramid.data_ptr(), coords_rows.data_ptr(), B, H, W, self.q_count, self.num_levels,
                    self.radius, corr.data_ptr(), qmax.data_ptr(), _lib.stream_of(out)),
                    "RowShardedCorrBlock lookup (split convc1)")
                _lib.check(_lib.lib().ecorr_conv1x1_relu_split(
                    corr.data_ptr(), B, C, self.q_count, qmax.data_ptr(), G, wt.data_ptr(),
                    None if bias is None else bias.data_ptr(), O, out.data_ptr(), _lib.stream_of(out)),
                    "RowShardedCorrBlock lookup+conv1x1+relu (split)")
                return out if self.world == 1 else self._ex.gather(B, O, W, self._device)
            wt = _lib.packed_conv1x1_weight(weight, O, C, "fused", _lib.stream_of(out), self._wcache)
            _lib.check(_lib.lib().ecorr_lookup_conv1x1_relu_packed(
                self._pyramid.data_ptr(), coords_rows.data_ptr(), B, H, W, self.q_count, self.num_levels,
                self.radius, wt.data_ptr(), None if bias is None else bias.data_ptr(), O, out.data_ptr(),
                _lib.stream_of(out)), "RowShardedCorrBlock lookup+conv1x1+relu")
        if self.world == 1:
            return out
        return self._ex.gather(B, O, W, self._device)                        # exchange 2 (fused)
