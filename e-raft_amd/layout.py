"""Tiled pyramid storage (include/ecorr.h): each query image of level i is stored as row-major
4 x 8-float tiles (128 bytes).  `untile` turns a level back into the reference's corr_pyramid
shape [rows, 1, h, w] (a copy; nothing on the E-RAFT path reads corr_pyramid, corr.py:16-27);
`tile` is the inverse, used to feed externally produced pyramids (tests) to ecorr_lookup."""
import torch

TILE_H, TILE_W = 4, 8


def padded(h, w):
    return -(-h // TILE_H) * TILE_H, -(-w // TILE_W) * TILE_W


def untile(flat, rows, h, w):
    """flat level storage -> [rows, 1, h, w] contiguous tensor in the reference layout."""
    hp, wp = padded(h, w)
    t = flat.view(rows, hp // TILE_H, wp // TILE_W, TILE_H, TILE_W).permute(0, 1, 3, 2, 4)
    return t.reshape(rows, hp, wp)[:, :h, :w].contiguous().view(rows, 1, h, w)


def tile(level):
    """[rows, h, w] (or [rows, 1, h, w]) reference-layout level -> flat tiled storage (zero pad)."""
    level = torch.as_tensor(level)
    rows, h, w = level.shape[0], level.shape[-2], level.shape[-1]
    hp, wp = padded(h, w)
    buf = level.new_zeros((rows, hp, wp))
    buf[:, :h, :w] = level.reshape(rows, h, w)
    return buf.view(rows, hp // TILE_H, TILE_H, wp // TILE_W, TILE_W).permute(0, 1, 3, 2, 4).reshape(-1)
