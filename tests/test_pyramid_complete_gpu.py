"""Every pyramid element is written by the build (a store that silently drops would hide
behind an allocation reused from an identical earlier build).

The pyramid allocation is pre-filled with a NaN of a payload no build produces (0x7fc0dead), then
built from finite fmaps through the C ABI (ecorr_build_split / ecorr_build); every element of every
level in the reference layout must be overwritten -- finite, and never that payload.  Shapes: the
DSEC bench shape (FULL 256-query tiles whose first row starts a 64-row interleave group, plus the
partial last tile), ragged maps (non-FULL tiles, band n-tiles, padded tile rows), and a query-row
slab whose first row is not group-aligned.
"""
import ctypes

import numpy as np
import pytest
import torch

import prng

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SENTINEL = 0x7FC0DEAD


@pytest.fixture(scope="module")
def ea():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


CASES = [  # (B, D, H, W, slab row0, slab rows or None = whole map, levels)
    (16, 256, 60, 80, 0, None, 4),     # bench C2: FULL tiles + the partial last one, band n-tiles (H % 8 = 4)
    (3, 256, 23, 40, 0, None, 4),      # ragged: H % 8 = 7 (padded regular tile row), 920 queries
    (2, 256, 19, 30, 0, None, 4),      # H % 8 = 3 (band), W % 16 = 14
    (2, 256, 30, 40, 7, 9, 4),         # query-row slab starting mid-group (rows 7..15)
    (1, 100, 17, 22, 0, None, 3),      # D != 256: the 32x32x16 split kernel
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b%d_d%d_%dx%d_r%d_%s" % (c[:5] + (c[5] or "all",)))
@pytest.mark.parametrize("mode", ["split", "fp32"])
def test_every_element_written(ea, case, mode):
    from eraft_amd import _lib
    from eraft_amd.layout import formats, untile
    B, D, H, W, r0, rr, L = case
    f1n = prng.normal(7 + H, (B, D, H, W))
    f2n = prng.normal(8 + W, (B, D, H, W))
    if rr is not None:
        f1n = np.ascontiguousarray(f1n[:, :, r0:r0 + rr])
    q = (rr if rr is not None else H) * W
    f1, f2 = torch.from_numpy(f1n).to(DEV), torch.from_numpy(f2n).to(DEV)
    h, w, off = _lib.layout(B * q, H, W, L)
    pyr = torch.full((off[-1],), 0, dtype=torch.int32, device=DEV).fill_(SENTINEL).view(torch.float32)
    st = _lib.stream_of(f2)
    with torch.no_grad():
        if mode == "split":
            nb = ctypes.c_int64()
            _lib.check(_lib.lib().ecorr_build_split_workspace_size(B, D, H, W, q, ctypes.byref(nb)), "ws")
            ws = torch.empty(nb.value, dtype=torch.uint8, device=DEV)
            _lib.check(_lib.lib().ecorr_build_split(f1.data_ptr(), f2.data_ptr(), B, D, H, W, q, L, pyr.data_ptr(),
                                                    ws.data_ptr(), st), "split build")
        else:
            _lib.check(_lib.lib().ecorr_build(f1.data_ptr(), f2.data_ptr(), B, D, H, W, q, L, pyr.data_ptr(), st),
                       "fp32 build")
        torch.cuda.synchronize()
    ntx = formats(H, W, L)
    for i in range(L):
        lv = untile(pyr[off[i]:off[i + 1]], B * q, h[i], w[i], ntx[i], i)
        bits = lv.contiguous().view(torch.int32)
        missing = int((bits == SENTINEL).sum())
        assert missing == 0, f"level {i}: {missing} of {lv.numel()} elements never written"
        assert bool(torch.isfinite(lv).all()), f"level {i}: non-finite values from finite fmaps"
