"""Query-row sharded CorrBlock for high-resolution frames (BASELINE configs[4]).

The all-pairs volume row of query pixel p depends only on fmap1[:, :, p] and ALL of fmap2, and
the pyramid pools over fmap2's (target) dims.  So the query pixels split cleanly by image rows:
rank r owns rows [start_r, start_r + rows_r) of the 1/8-resolution map, builds the pyramid for
those queries only (1/world of the GEMM and of the 1.15 GB/pair volume at 1280x720), and answers
lookups for them with no communication.  The exchanges are:

  1. fmap2 all-gather, once per frame pair, when the feature maps arrive as row slabs (a
     spatially sharded fnet): RowShardedCorrBlock.from_row_slabs;
  2. lookup-output all-gather, once per GRU iteration, because ERAFT.forward keeps the GRU
     replicated and needs the full [B, 324, H, W] on every rank (eraft.py:128-132).

Both are one collective each over the process group (RCCL over xGMI with the "nccl" backend; any
backend works, the CPU tests use gloo).  Ragged row counts (92 rows over 8 ranks = 12,12,12,12,
11,11,11,11) are padded to the largest slab for the collective and cropped when reassembled.
"""
import torch
import torch.distributed as dist

from . import _lib
from .corr import _no_grad_inputs, _require_device_f32
from .layout import formats, untile


def row_partition(H, world):
    """Contiguous near-equal row blocks: (starts, counts), counts differ by at most one."""
    if world < 1 or H < world:
        raise ValueError(f"cannot split {H} rows over {world} ranks")
    base, extra = divmod(H, world)
    counts = [base + (1 if r < extra else 0) for r in range(world)]
    starts = [sum(counts[:r]) for r in range(world)]
    return starts, counts


def gather_rows(slab, counts, group=None):
    """All-gather per-rank row slabs [..., rows_r, W] into the full [..., sum(rows), W].

    Slabs are zero-padded to max(counts) rows so one fixed-size collective serves ragged splits.
    """
    world = dist.get_world_size(group)
    if world == 1:
        return slab.contiguous()
    maxr = max(counts)
    lead = slab.shape[:-2]
    W = slab.shape[-1]
    if slab.shape[-2] != maxr:
        pad = slab.new_zeros(*lead, maxr, W)
        pad[..., :slab.shape[-2], :] = slab
    else:
        pad = slab.contiguous()
    if dist.get_backend(group) == "nccl":
        buf = slab.new_empty((world,) + tuple(pad.shape))
        dist.all_gather_into_tensor(buf, pad, group=group)
        parts = [buf[r] for r in range(world)]
    else:
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
    return torch.cat([parts[r][..., :counts[r], :] for r in range(world)], dim=-2).contiguous()


class RowShardedCorrBlock:
    """CorrBlock over a process group, queries sharded by image rows.

    RowShardedCorrBlock(fmap1, fmap2, ...)            full fmaps on every rank (replicated fnet);
    RowShardedCorrBlock.from_row_slabs(f1_rows, f2_rows, H, ...)   row slabs, fmap2 all-gathered.
    __call__(coords) takes the full [B, 2, H, W] coords (replicated GRU) and returns the full
    [B, C, H, W] lookup on every rank, bit-identical to the unsharded CorrBlock.
    """

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        _require_device_f32("fmap1", fmap1)
        B, D, H, W = fmap1.shape
        self.starts, self.counts = row_partition(H, self.world)
        r0, rr = self.starts[self.rank], self.counts[self.rank]
        self._init_local(fmap1[:, :, r0:r0 + rr].contiguous(), fmap2.contiguous(), num_levels, radius)

    @classmethod
    def from_row_slabs(cls, fmap1_rows, fmap2_rows, H, num_levels=4, radius=4, group=None):
        self = cls.__new__(cls)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.starts, self.counts = row_partition(H, self.world)
        if fmap1_rows.shape[2] != self.counts[self.rank] or fmap2_rows.shape != fmap1_rows.shape:
            raise RuntimeError(f"rank {self.rank}: row slabs {tuple(fmap1_rows.shape)} / "
                               f"{tuple(fmap2_rows.shape)} do not match {self.counts[self.rank]} rows")
        fmap2 = gather_rows(fmap2_rows.contiguous(), self.counts, group)   # exchange 1
        self._init_local(fmap1_rows.contiguous(), fmap2, num_levels, radius)
        return self

    def _init_local(self, fmap1_rows, fmap2, num_levels, radius):
        _require_device_f32("fmap1", fmap1_rows)
        _require_device_f32("fmap2", fmap2)
        _no_grad_inputs(fmap1_rows, fmap2)
        self.num_levels, self.radius = num_levels, radius
        B, D, H, W = fmap2.shape
        self._shape = (B, D, H, W)
        self._device = fmap2.device
        self.q_count = self.counts[self.rank] * W
        self._h, self._w, self._off = _lib.layout(B * self.q_count, H, W, num_levels)
        with torch.cuda.device(self._device):
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
                untile(self._pyramid[self._off[i]:self._off[i + 1]], rows, self._h[i], self._w[i], ntx[i])
                for i in range(self.num_levels)]
        return self._levels_cache

    def lookup_local(self, coords_rows):
        """Lookup for this rank's query rows: coords [B, 2, rows_r, W] -> [B, C, rows_r, W]."""
        B, _, H, W = self._shape
        rr = self.counts[self.rank]
        _require_device_f32("coords", coords_rows)
        if tuple(coords_rows.shape) != (B, 2, rr, W):
            raise RuntimeError(f"coords rows {tuple(coords_rows.shape)} != {(B, 2, rr, W)}")
        coords_rows = coords_rows.contiguous()
        K = 2 * self.radius + 1
        C = self.num_levels * K * K
        with torch.cuda.device(self._device):
            out = torch.empty((B, C, rr, W), dtype=torch.float32, device=self._device)
            _lib.check(_lib.lib().ecorr_lookup(
                self._pyramid.data_ptr(), coords_rows.data_ptr(), B, H, W, self.q_count,
                self.num_levels, self.radius, out.data_ptr(), _lib.stream_of(out)),
                "RowShardedCorrBlock lookup")
        return out

    def __call__(self, coords):
        B, _, H, W = self._shape
        if tuple(coords.shape) != (B, 2, H, W):
            raise RuntimeError(f"coords shape {tuple(coords.shape)} != {(B, 2, H, W)}")
        r0, rr = self.starts[self.rank], self.counts[self.rank]
        local = self.lookup_local(coords[:, :, r0:r0 + rr])
        return gather_rows(local, self.counts, self.group)                 # exchange 2
