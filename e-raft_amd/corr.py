"""Drop-in CorrBlock for E-RAFT on MI355X (mirrors /root/reference/model/corr.py).

Same constructor and call signatures as the reference:
    corr_fn = CorrBlock(fmap1, fmap2, num_levels=4, radius=4)      # corr.py:13  (eraft.py:107)
    corr    = corr_fn(coords1)                                       # corr.py:29  (eraft.py:128)
    CorrBlock.corr(fmap1, fmap2) -> [B, H, W, 1, H, W]               # corr.py:52
    corr_fn.corr_pyramid[i] : [B*H*W, 1, h_i, w_i]                   # corr.py:16,24,27
The work happens in libecorr.so (hand-written gfx950 HIP kernels, C ABI include/ecorr.h): one
MFMA GEMM launch builds all 4 pyramid levels, one gather launch serves each lookup.  No ATen
compute op runs on the hot path and there is no CPU fallback.  The pyramid lives in a tiled,
gather-friendly layout (layout.py); corr_pyramid materializes the reference-layout levels on
first access (nothing on the E-RAFT path reads it).

Contract differences, all loud: inputs must be fp32 HIP tensors (the reference path is fp32,
eraft.py:104-105); the block is forward-only (E-RAFT only ever calls it under torch.no_grad(),
test.py:80) and refuses inputs that require grad while grad mode is on; coords must match the
build's (B, 2, H, W) exactly.

Numerics: the default build sums each product as f16 lo*hi + hi*lo + hi*hi of per-pixel-scaled
operands: within 1e-5 normwise of the reference and closer to fp64 than its fp32
GEMM, pooling and lookup bit-exact given level 0.  One semantic difference: an fmap pixel holding
+-inf yields NaN (not +-inf) in its level-0 row/column, because the lo half of an infinite value
is NaN; NaN inputs give NaN in both.  ECORR_BUILD_MODE=fp32 (read once at import) selects the
fp32-MFMA build, which keeps the reference's inf semantics.

corr_pyramid is a materialized COPY in the reference layout: 4 levels of B*H*W query images
(1.96 GB at DSEC B=16, the whole pyramid again), made on first access and cached on the block.
Nothing on the E-RAFT path reads it; access it only for inspection or tests.
"""
import ctypes
import os
import weakref

import torch

from . import _lib
from .layout import formats, untile


def _require_device_f32(name, t):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} is on {t.device}: eraft_amd runs only on HIP devices (no CPU path)")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")


def _version(t):
    try:
        return t._version
    except RuntimeError:   # inference tensor: no version counter (and no in-place updates)
        return -1


def _no_grad_inputs(*ts):
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        raise RuntimeError("eraft_amd CorrBlock is forward-only; call it under torch.no_grad() "
                           "(as the reference harness does, test.py:80)")


class CorrBlock:
    """All-pairs correlation pyramid + radius-r lookup (reference: model/corr.py:12-60)."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels = num_levels
        self.radius = radius
        _require_device_f32("fmap1", fmap1)
        _require_device_f32("fmap2", fmap2)
        _no_grad_inputs(fmap1, fmap2)
        if fmap1.dim() != 4 or fmap1.shape != fmap2.shape:
            raise RuntimeError(f"fmap shapes {tuple(fmap1.shape)} / {tuple(fmap2.shape)} differ "
                               "or are not [B, D, H, W]")
        if fmap1.device != fmap2.device:
            raise RuntimeError("fmap1 and fmap2 are on different devices")
        if not (fmap1.is_contiguous() and fmap2.is_contiguous()):
            # the reference .view()s them (corr.py:55-56), which raises on these strides
            raise RuntimeError("fmap1/fmap2 must be contiguous (reference: view size is not "
                               "compatible with input tensor's size and stride)")
        B, D, H, W = fmap1.shape
        # degenerate shapes as the reference (tests/golden/degenerate.npz): an empty batch or map
        # raises where its reshape / avg_pool2d do (corr.py:16-24); D = 0 feature channels give
        # 0 / sqrt(0) = NaN volumes, which its lookup samples like any other values
        if B == 0:
            raise RuntimeError(f"cannot reshape tensor of 0 elements into shape [0, {H}, {W}, -1] "
                               "(empty batch: the reference's CorrBlock.corr reshape)")
        if H == 0 or W == 0:
            raise RuntimeError(f"Expected 3D or 4D (batch mode) tensor with optional 0 dim batch size for "
                               f"input, but got:[{B * H * W}, 1, {H}, {W}] (empty map: the reference's avg_pool2d)")
        self._shape = (B, D, H, W)
        self._device = fmap1.device
        Q = H * W
        self._h, self._w, self._off = _lib.layout(B * Q, H, W, num_levels)
        with _lib.on_device(self._device):
            if D == 0:
                self._pyramid = torch.full((self._off[-1],), float("nan"), dtype=torch.float32, device=self._device)
            else:
                self._pyramid = _lib.build_pyramid(fmap1, fmap2, B, D, H, W, Q, num_levels, self._off,
                                                   "CorrBlock build")
        self._rows = B * Q
        self._levels_cache = None
        self._wcache = {}   # packed convc1 weights of this block (_lib.packed_conv1x1_weight)
        # presplit convc1: the column scales come from the fmaps (ecorr_split_column_scale), computed
        # on the first presplit call; weak references and version counters, so the block neither
        # keeps the fmaps alive nor trusts them after an in-place change (then: the split mode)
        self._fmap_refs = (weakref.ref(fmap1), weakref.ref(fmap2), _version(fmap1), _version(fmap2))
        self._colscale = None

    @property
    def corr_pyramid(self):
        """Reference-layout levels [B*H*W, 1, h_i, w_i] (corr.py:16-27), materialized on demand."""
        if self._levels_cache is None:
            ntx = formats(self._shape[2], self._shape[3], self.num_levels)
            self._levels_cache = [
                untile(self._pyramid[self._off[i]:self._off[i + 1]], self._rows, self._h[i], self._w[i],
                       ntx[i], i)
                for i in range(self.num_levels)]
        return self._levels_cache

    def __call__(self, coords):
        B, _, H, W = self._shape
        _require_device_f32("coords", coords)
        _no_grad_inputs(coords)
        if tuple(coords.shape) != (B, 2, H, W):
            raise RuntimeError(f"coords shape {tuple(coords.shape)} != {(B, 2, H, W)} of the pyramid")
        if coords.device != self._device:
            raise RuntimeError("coords is on a different device than the pyramid")
        coords = coords.contiguous()   # the reference accepts any strides (permute + reshape)
        K = 2 * self.radius + 1
        C = self.num_levels * K * K
        with _lib.on_device(self._device):
            out = torch.empty((B, C, H, W), dtype=torch.float32, device=self._device)
            _lib.check(_lib.lib().ecorr_lookup(
                self._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, self.num_levels,
                self.radius, out.data_ptr(), _lib.stream_of(coords)), "CorrBlock lookup")
        return out

    def lookup_conv1x1_relu(self, coords, weight, bias=None, mode=None):
        """F.relu(conv1x1(self(coords), weight, bias)): the lookup followed by
        BasicMotionEncoder.convc1 + ReLU (update.py:67,74).
        weight: [O, C, 1, 1] (or [O, C]) fp32 with C = num_levels * (2r+1)^2; bias: [O] or None.
        Returns [B, O, H, W].  mode (default: env ECORR_CONVC1, else "split"):
          "split"  ecorr_lookup_qmax into a temporary [B, C, H, W] (+ per-query maxima), then
                   ecorr_conv1x1_relu_split (f16 matrix cores, split operands: normwise within 1e-5
                   of the fp32 conv);
          "presplit" (ABI 16, radius 4, <= 4 levels) ecorr_lookup_presplit writes corr already split
                   (f16 hi + lo under a per-query bound scale from the fmaps, ecorr_split_column_scale,
                   once per block) and ecorr_conv1x1_relu_presplit loads it whole: normwise within 1e-5;
                   falls back to "split" when the fmaps are gone or changed in place since the build;
                   measured no faster than "split" (DESIGN.md §3.3);
          "fused"  ecorr_lookup_conv1x1_relu_packed: one kernel, the lookup tile never leaves the
                   CU, an exact c-ordered fp32 MFMA sum (radius 4, num_levels <= 4, O a multiple of 64)."""
        mode = mode or os.environ.get("ECORR_CONVC1", "split")
        if mode not in ("split", "presplit", "fused"):
            raise ValueError(f"mode {mode!r}: expected 'split', 'presplit' or 'fused'")
        B, _, H, W = self._shape
        _require_device_f32("coords", coords)
        _require_device_f32("weight", weight)
        _no_grad_inputs(coords, weight, *(() if bias is None else (bias,)))
        if tuple(coords.shape) != (B, 2, H, W):
            raise RuntimeError(f"coords shape {tuple(coords.shape)} != {(B, 2, H, W)} of the pyramid")
        if any(t.device != self._device for t in (coords, weight, *(() if bias is None else (bias,)))):
            raise RuntimeError("coords / weight / bias are on a different device than the pyramid")
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
        coords = coords.contiguous()
        bptr = None if bias is None else bias.data_ptr()
        with _lib.on_device(self._device):
            out = torch.empty((B, O, H, W), dtype=torch.float32, device=self._device)
            st = _lib.stream_of(coords)
            if mode == "presplit":
                scale = self._column_scale(st) if self.radius == 4 and self.num_levels <= 4 else None
                if scale is None:
                    mode = "split"
            if mode == "presplit":
                wt = _lib.packed_conv1x1_weight(weight, O, C, "presplit", st, self._wcache)   # once per block
                nbytes = ctypes.c_int64()
                _lib.check(_lib.lib().ecorr_presplit_size(B, self.num_levels, H * W, ctypes.byref(nbytes)),
                           "CorrBlock presplit size")
                corr = torch.empty(nbytes.value, dtype=torch.uint8, device=self._device)
                _lib.check(_lib.lib().ecorr_lookup_presplit(
                    self._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, self.num_levels, self.radius,
                    scale.data_ptr(), corr.data_ptr(), st), "CorrBlock lookup (presplit convc1)")
                _lib.check(_lib.lib().ecorr_conv1x1_relu_presplit(
                    corr.data_ptr(), B, self.num_levels, H * W, scale.data_ptr(), wt.data_ptr(), bptr, O,
                    out.data_ptr(), st), "CorrBlock lookup+conv1x1+relu (presplit)")
            elif mode == "split":
                wt = _lib.packed_conv1x1_weight(weight, O, C, "split", st, self._wcache)   # once per block
                G = 3 * self.num_levels
                corr = torch.empty((B, C, H, W), dtype=torch.float32, device=self._device)
                qmax = torch.empty((B, G, H * W), dtype=torch.float32, device=self._device)
                _lib.check(_lib.lib().ecorr_lookup_qmax(
                    self._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, self.num_levels, self.radius,
                    corr.data_ptr(), qmax.data_ptr(), st), "CorrBlock lookup (split convc1)")
                _lib.check(_lib.lib().ecorr_conv1x1_relu_split(
                    corr.data_ptr(), B, C, H * W, qmax.data_ptr(), G, wt.data_ptr(), bptr, O, out.data_ptr(), st),
                    "CorrBlock lookup+conv1x1+relu (split)")
            else:
                wt = _lib.packed_conv1x1_weight(weight, O, C, "fused", st, self._wcache)   # once per block
                _lib.check(_lib.lib().ecorr_lookup_conv1x1_relu_packed(
                    self._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, self.num_levels,
                    self.radius, wt.data_ptr(), bptr, O, out.data_ptr(), st), "CorrBlock lookup+conv1x1+relu")
        return out

    def _column_scale(self, st):
        """int[B*H*W + B]: the presplit column exponents (ecorr_split_column_scale), once per block;
        None when the fmaps are gone or were changed in place since the build."""
        if self._colscale is None:
            r1, r2, v1, v2 = self._fmap_refs
            f1, f2 = r1(), r2()
            if f1 is None or f2 is None or _version(f1) != v1 or _version(f2) != v2:
                return None
            B, D, H, W = self._shape
            sc = torch.empty(B * H * W + B, dtype=torch.int32, device=self._device)
            _lib.check(_lib.lib().ecorr_split_column_scale(f1.data_ptr(), f2.data_ptr(), B, D, H, W, sc.data_ptr(),
                                                           st), "CorrBlock presplit column scale")
            self._colscale = sc
            self._fmap_refs = None
        return self._colscale

    @staticmethod
    def corr(fmap1, fmap2):
        """Level-0 volume fmap1^T fmap2 / sqrt(D) as [B, H, W, 1, H, W] (corr.py:52-60)."""
        blk = CorrBlock(fmap1, fmap2, num_levels=1, radius=0)
        B, _, H, W = fmap1.shape
        return blk.corr_pyramid[0].view(B, H, W, 1, H, W)
