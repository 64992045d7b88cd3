"""Pyramid storage (include/ecorr.h).  Each query image of level i is stored either as row-major
4 x 8-float tiles (128 bytes, one L2 line) or, for small levels >= 2 where tile padding would
exceed half the image, compact row-major; `formats` asks libecorr which (ntx = tiles per tile row,
0 = compact).  `untile` turns a level back into the reference's corr_pyramid shape
[rows, 1, h, w] (nothing on the E-RAFT path reads corr_pyramid, corr.py:16-27); `tile` and `pack`
are the inverse, used to feed externally produced pyramids (tests) to ecorr_lookup."""
import ctypes

import torch

from . import _lib

TILE_H, TILE_W = 4, 8


def padded(h, w):
    return -(-h // TILE_H) * TILE_H, -(-w // TILE_W) * TILE_W


def formats(H, W, levels):
    """ntx per level: tiles per tile row, or 0 for a compact row-major level."""
    ntx = (ctypes.c_int * levels)()
    _lib.check(_lib.lib().ecorr_pyramid_formats(H, W, levels, ntx), "CorrBlock pyramid")
    return list(ntx)


def untile(flat, rows, h, w, ntx):
    """flat level storage -> [rows, 1, h, w] tensor in the reference layout (a view when the
    level is compact, a copy when tiled)."""
    if ntx == 0:
        return flat[:rows * h * w].view(rows, 1, h, w)
    hp, wp = padded(h, w)
    t = flat[:rows * hp * wp].view(rows, hp // TILE_H, wp // TILE_W, TILE_H, TILE_W).permute(0, 1, 3, 2, 4)
    return t.reshape(rows, hp, wp)[:, :h, :w].contiguous().view(rows, 1, h, w)


def tile(level, ntx=1):
    """[rows, h, w] (or [rows, 1, h, w]) reference-layout level -> flat storage (zero pad)."""
    level = torch.as_tensor(level)
    rows, h, w = level.shape[0], level.shape[-2], level.shape[-1]
    if ntx == 0:
        return level.reshape(-1).contiguous()
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
        t = tile(torch.as_tensor(lv), ntx[i])
        buf[off[i]:off[i] + t.numel()] = t
    return buf
