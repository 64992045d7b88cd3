"""Pyramid storage (include/ecorr.h).  Each query image of level 0 (and >= 4) is stored as
row-major 4 x 8-float tiles (128 bytes, one L2 line) or, for small levels >= 4 where tile padding
would exceed half the image, compact row-major; levels 1-3 are interleaved: query rows in groups
of 64, each group storing every 2 x 4 (levels 1-2) / 1 x 2 (level 3) block of the level for its 64
rows back to back.  `formats` asks libecorr which (ntx = tiles per tile row, 0 = compact, -nbx =
interleaved with nbx blocks per block row).  `untile` turns a level back into the reference's
corr_pyramid shape [rows, 1, h, w] (nothing on the E-RAFT path reads corr_pyramid,
corr.py:16-27); `tile` and `pack` are the inverse, used to feed externally produced pyramids
(tests) to ecorr_lookup."""
import ctypes

import torch

from . import _lib

TILE_H, TILE_W = 4, 8


def padded(h, w):
    return -(-h // TILE_H) * TILE_H, -(-w // TILE_W) * TILE_W


GROUP = 64   # query rows per interleave group (ecorr_device.h kGroup)


def block_shape(level):
    """(bh, bw) of an interleaved level's blocks (include/ecorr.h): 2 x 4 at levels 1-2, 1 x 2 at 3."""
    assert level in (1, 2, 3), level
    return (1, 2) if level == 3 else (2, 4)


def formats(H, W, levels):
    """ntx per level: tiles per tile row, 0 for a compact row-major level, -nbx for an
    interleaved level (nbx blocks per block row)."""
    ntx = (ctypes.c_int * levels)()
    _lib.check(_lib.lib().ecorr_pyramid_formats(H, W, levels, ntx), "CorrBlock pyramid")
    return list(ntx)


def untile(flat, rows, h, w, ntx, level=None):
    """flat level storage -> [rows, 1, h, w] tensor in the reference layout (a view when the
    level is compact, a copy when tiled or interleaved; interleaved levels need `level`)."""
    if ntx == 0:
        return flat[:rows * h * w].view(rows, 1, h, w)
    if ntx < 0:
        bh, bw = block_shape(level)
        nbx, nby = -ntx, -(-h // bh)
        ng = -(-rows // GROUP)
        t = flat[:ng * nby * nbx * GROUP * bh * bw].view(ng, nby, nbx, GROUP, bh, bw).permute(0, 3, 1, 4, 2, 5)
        return t.reshape(ng * GROUP, nby * bh, nbx * bw)[:rows, :h, :w].contiguous().view(rows, 1, h, w)
    hp, wp = padded(h, w)
    t = flat[:rows * hp * wp].view(rows, hp // TILE_H, wp // TILE_W, TILE_H, TILE_W).permute(0, 1, 3, 2, 4)
    return t.reshape(rows, hp, wp)[:, :h, :w].contiguous().view(rows, 1, h, w)


def tile(level, ntx=1, index=None):
    """[rows, h, w] (or [rows, 1, h, w]) reference-layout level -> flat storage (zero pad);
    interleaved formats (ntx < 0) need the level's `index`."""
    level = torch.as_tensor(level)
    rows, h, w = level.shape[0], level.shape[-2], level.shape[-1]
    if ntx == 0:
        return level.reshape(-1).contiguous()
    if ntx < 0:
        bh, bw = block_shape(index)
        nbx, nby = -ntx, -(-h // bh)
        ng = -(-rows // GROUP)
        buf = level.new_zeros((ng * GROUP, nby * bh, nbx * bw))
        buf[:rows, :h, :w] = level.reshape(rows, h, w)
        return buf.view(ng, GROUP, nby, bh, nbx, bw).permute(0, 2, 4, 1, 3, 5).reshape(-1)
    hp, wp = padded(h, w)
    buf = level.new_zeros((rows, hp, wp))
    buf[:, :h, :w] = level.reshape(rows, h, w)
    return buf.view(rows, hp // TILE_H, TILE_H, wp // TILE_W, TILE_W).permute(0, 1, 3, 2, 4).reshape(-1)


def pack(levels, H, W):
    """Reference-layout levels ([rows, h, w] each, level 0 = H x W) -> the flat pyramid buffer
    ecorr_lookup reads, at the library's level offsets."""
    rows = levels[0].shape[0]
    n = len(levels)
    _, _, off = _lib.layout(rows, H, W, n)
    ntx = formats(H, W, n)
    buf = torch.zeros(off[-1], dtype=torch.float32)
    for i, lv in enumerate(levels):
        t = tile(torch.as_tensor(lv), ntx[i], i)
        buf[off[i]:off[i] + t.numel()] = t
    return buf


def levels_of(pyramid, rows, H, W, levels):
    """The flat pyramid of `rows` query rows -> reference-layout levels [rows, 1, h_i, w_i]."""
    h, w, off = _lib.layout(rows, H, W, levels)
    ntx = formats(H, W, levels)
    return [untile(pyramid[off[i]:off[i + 1]], rows, h[i], w[i], ntx[i], i) for i in range(levels)]
