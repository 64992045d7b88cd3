"""CPU-side checks of the C ABI: the library builds for gfx950, loads, exports every symbol the
header declares, and validates arguments before touching a device (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ecorr.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ecorr_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def ea():
    lib = os.path.join(ROOT, "e-raft_amd", "libecorr.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "e-raft_amd", "csrc")], check=True)
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


def test_header_symbols_exported(ea):
    names = _declared()
    assert {"ecorr_build", "ecorr_lookup", "ecorr_pyramid_layout", "ecorr_bilinear_sampler",
            "ecorr_coords_grid", "ecorr_strerror", "ecorr_abi_version"} <= set(names)
    L = ctypes.CDLL(ea.LIB_PATH)
    for n in names:
        assert hasattr(L, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", ea.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (ecorr_\w+)", out))
    assert exported == set(names)


def test_library_reads_no_environment(ea):
    """No runtime knobs: the library imports no getenv/secure_getenv, so a stray variable cannot
    change a result (round 1 read ECORR_BUILD_SKIP_EPILOGUE & co. on every launch)."""
    out = subprocess.run(["nm", "-D", "--undefined-only", ea.LIB_PATH], capture_output=True, text=True).stdout
    assert not re.search(r"\bU (secure_)?getenv\b", out), out
    for src in sorted(os.listdir(os.path.join(ROOT, "e-raft_amd", "csrc"))):
        if src.endswith((".hip", ".h")):
            assert "getenv" not in open(os.path.join(ROOT, "e-raft_amd", "csrc", src)).read(), src


def test_code_object_is_gfx950(ea):
    # the embedded HIP fat binary names its offload targets (amdgcn-amd-amdhsa--gfx950)
    data = open(ea.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-+(gfx\w+)", data))
    assert targets == {b"gfx950"}


def test_layout_matches_reference_shapes(ea):
    from eraft_amd import _lib
    h, w, off = _lib.layout(16 * 4800, 60, 80, 4)
    assert (h, w) == ([60, 30, 15, 7], [80, 40, 20, 10])
    # level 0 tiled (each image 4 x 8 tiles: 60x80 exactly); levels 1-3 interleaved in 2 x 4 / 2 x 4
    # / 1 x 2 blocks (30 x 40 -> 15 x 10 blocks, 15 x 20 -> 8 x 5, 7 x 10 -> 7 x 5); every level
    # starts on a 128-byte line
    sizes = [60 * 80, 15 * 10 * 8, 8 * 5 * 8, 7 * 5 * 2]
    assert off == [0] + list(np.cumsum([76800 * s for s in sizes]))
    from eraft_amd.layout import formats
    assert formats(60, 80, 4) == [10, -10, -5, -5]
    assert formats(32, 32, 4) == [4, -4, -2, -2]      # MVSEC: 16 x 16, 8 x 8 and 4 x 4 levels
    assert formats(92, 160, 4) == [20, -20, -10, -10]  # 1280x720: 46 x 80, 23 x 40 and 11 x 20 levels
    # 3 rows: interleaved levels hold whole 64-row groups (10x10 -> 5 x 3 blocks of 8, 5x5 -> 3 x 2
    # blocks of 8, 2x2 -> 2 x 1 of 2)
    _, _, off = _lib.layout(3, 20, 20, 4)
    assert formats(20, 20, 4) == [3, -3, -2, -1]
    assert off == [0, 1440, 1440 + 64 * 120, 1440 + 64 * 120 + 64 * 48, 1440 + 64 * 120 + 64 * 48 + 64 * 4]
    # levels past 3 stay tiled, or compact where tiles would pad them by more than half
    assert formats(64, 64, 6) == [8, -8, -4, -4, 0, 0]
    assert formats(128, 256, 6) == [32, -32, -16, -16, 2, 1]
    th, tw = ctypes.c_int(), ctypes.c_int()
    assert ea.lib().ecorr_pyramid_tile(ctypes.byref(th), ctypes.byref(tw)) == 0
    assert (th.value, tw.value) == (4, 8)
    h, w, _ = _lib.layout(396, 18, 22, 4)
    assert (h, w) == ([18, 9, 4, 2], [22, 11, 5, 2])


@pytest.mark.parametrize("hw", [(4, 4), (2, 40), (6, 6)])
def test_zero_level_raises_like_reference(ea, hw):
    from eraft_amd import _lib
    with pytest.raises(RuntimeError, match="too small"):
        _lib.layout(hw[0] * hw[1], hw[0], hw[1], 4)


def test_argument_validation_before_launch(ea):
    L = ea.lib()
    from eraft_amd import _lib
    assert L.ecorr_build(None, None, 1, 256, 8, 8, 64, 4, None, None) == _lib.ECORR_EINVAL
    # q_count outside [1, H*W]
    assert L.ecorr_build(8, 8, 1, 256, 8, 8, 65, 4, 8, None) == _lib.ECORR_EINVAL
    assert L.ecorr_build(8, 8, 1, 256, 8, 8, 0, 4, 8, None) == _lib.ECORR_EINVAL
    assert L.ecorr_lookup(8, 8, 1, 8, 8, 64, 4, 33, 8, None) == _lib.ECORR_ERADIUS
    assert L.ecorr_lookup(8, 8, 1, 8, 8, 64, 0, 4, 8, None) == _lib.ECORR_ELEVELS
    assert L.ecorr_lookup(8, 8, 1, 4, 4, 16, 4, 4, 8, None) == _lib.ECORR_ESHAPE
    assert "too small" in _lib.strerror(_lib.ECORR_ESHAPE)
    # fused lookup + convc1: radius 4 / <= 4 levels only, O a multiple of 64, weight required
    F = L.ecorr_lookup_conv1x1_relu
    assert F(8, 8, 1, 16, 16, 256, 4, 3, 8, None, 64, 8, None) == _lib.ECORR_ERADIUS
    assert F(8, 8, 1, 64, 64, 4096, 5, 4, 8, None, 64, 8, None) == _lib.ECORR_ELEVELS   # levels > 4
    assert F(8, 8, 1, 16, 16, 256, 4, 4, 8, None, 96, 8, None) == _lib.ECORR_EINVAL
    assert F(8, 8, 1, 16, 16, 256, 4, 4, None, None, 64, 8, None) == _lib.ECORR_EINVAL
    Fp = L.ecorr_lookup_conv1x1_relu_packed   # ... with the packed weight (ABI 14)
    assert Fp(8, 8, 1, 16, 16, 256, 4, 3, 8, None, 64, 8, None) == _lib.ECORR_ERADIUS
    assert Fp(8, 8, 1, 16, 16, 256, 4, 4, 8, None, 96, 8, None) == _lib.ECORR_EINVAL
    assert Fp(8, 8, 1, 16, 16, 256, 4, 4, None, None, 64, 8, None) == _lib.ECORR_EINVAL
    n = ctypes.c_int64()
    assert L.ecorr_conv1x1_packed_size(256, 324, ctypes.byref(n)) == _lib.ECORR_OK
    assert n.value == 4 * 21 * 4 * 64 * 4   # [O / 64][ceil(C / 16)][4 pieces][64 lanes][4 floats]
    assert L.ecorr_conv1x1_packed_size(96, 324, ctypes.byref(n)) == _lib.ECORR_EINVAL
    assert L.ecorr_conv1x1_pack(None, 256, 324, 8, None) == _lib.ECORR_EINVAL
    assert L.ecorr_conv1x1_pack(8, 100, 324, 8, None) == _lib.ECORR_EINVAL
    # split-f16 convc1 + ReLU (ABI 15): [O/256 blocks][ceil(C/16) chunks][16 KB] + O-block exponents
    assert L.ecorr_conv1x1_split_size(256, 324, ctypes.byref(n)) == _lib.ECORR_OK
    assert n.value == 1 * 21 * 16384 + 256 * 4
    assert L.ecorr_conv1x1_split_size(300, 324, ctypes.byref(n)) == _lib.ECORR_OK
    assert n.value == 2 * 21 * 16384 + 512 * 4
    assert L.ecorr_conv1x1_split_size(0, 324, ctypes.byref(n)) == _lib.ECORR_EINVAL
    assert L.ecorr_conv1x1_split_pack(None, 256, 324, 8, None) == _lib.ECORR_EINVAL
    assert L.ecorr_conv1x1_split_pack(8, 256, 0, 8, None) == _lib.ECORR_EINVAL
    S = L.ecorr_conv1x1_relu_split   # (in, B, C, Q, qmax, G, packed, bias, O, out, stream)
    assert S(None, 1, 324, 4800, None, 0, 8, None, 256, 16, None) == _lib.ECORR_EINVAL
    assert S(8, 1, 324, 4800, None, 0, None, None, 256, 16, None) == _lib.ECORR_EINVAL
    assert S(8, 0, 324, 4800, None, 0, 8, None, 256, 16, None) == _lib.ECORR_EINVAL
    assert S(8, 1, 324, 4800, None, 0, 8, None, 256, 8, None) == _lib.ECORR_EINVAL   # in == out
    assert S(8, 1, 324, 1 << 20, None, 0, 8, None, 256, 16, None) == _lib.ECORR_EINVAL   # 32-bit offsets
    assert S(8, 1, 324, 4800, 24, 0, 8, None, 256, 16, None) == _lib.ECORR_EINVAL   # qmax without G
    # lookup + partial maxima: a qmax buffer is required, then validates like ecorr_lookup
    assert L.ecorr_lookup_qmax(8, 8, 1, 8, 8, 64, 4, 4, 8, None, None) == _lib.ECORR_EINVAL
    assert L.ecorr_lookup_qmax(8, 8, 1, 8, 8, 64, 4, 33, 8, 8, None) == _lib.ECORR_ERADIUS
    # the split build's stages validate like the whole call (no workspace / no operands)
    assert L.ecorr_build_split_pack(8, 8, 1, 256, 8, 8, 64, None, None) == _lib.ECORR_EINVAL
    assert L.ecorr_build_split_pack(None, 8, 1, 256, 8, 8, 64, 256, None) == _lib.ECORR_EINVAL
    assert L.ecorr_build_split_gemm(1, 256, 8, 8, 64, 4, 8, None, None) == _lib.ECORR_EINVAL
    assert L.ecorr_build_split_gemm(1, 256, 8, 8, 64, 4, None, 256, None) == _lib.ECORR_EINVAL
    assert L.ecorr_build_split_gemm(1, 256, 8, 8, 65, 4, 8, 256, None) == _lib.ECORR_EINVAL


def test_cpu_tensors_rejected_loudly(ea):
    import torch
    f = torch.zeros(1, 16, 8, 8)
    with pytest.raises(RuntimeError, match="HIP"):
        ea.CorrBlock(f, f)


def test_tile_untile_roundtrip():
    import torch
    from eraft_amd.layout import tile, untile
    for (h, w) in [(60, 80), (15, 20), (7, 10), (1, 1), (9, 11)]:
        lv = torch.arange(3 * h * w, dtype=torch.float32).reshape(3, h, w)
        flat = tile(lv, ntx=-(-w // 8))
        hp, wp = -(-h // 4) * 4, -(-w // 8) * 8
        assert flat.numel() == 3 * hp * wp
        assert torch.equal(untile(flat, 3, h, w, ntx=wp // 8)[:, 0], lv)
        compact = tile(lv, ntx=0)
        assert torch.equal(compact, lv.reshape(-1)) and torch.equal(untile(compact, 3, h, w, 0)[:, 0], lv)
        # element (y, x) of image r lives at r*hp*wp + ((y//4)*(wp//8) + x//8)*32 + (y%4)*8 + x%8
        r, y, x = 2, h - 1, w - 1
        assert flat[r * hp * wp + ((y // 4) * (wp // 8) + x // 8) * 32 + (y % 4) * 8 + x % 8] == lv[r, y, x]


def test_interleaved_roundtrip():
    """Levels 1-3: [64-row group][block][row][bh][bw] (include/ecorr.h), ragged rows and sides."""
    import torch
    from eraft_amd.layout import GROUP, tile, untile
    for level, (bh, bw) in ((1, (2, 4)), (2, (2, 4)), (3, (1, 2))):
        for rows, h, w in [(3, 15, 20), (130, 7, 10), (64, 1, 1), (65, 5, 9)]:
            lv = torch.arange(rows * h * w, dtype=torch.float32).reshape(rows, h, w)
            nbx, nby = -(-w // bw), -(-h // bh)
            flat = tile(lv, ntx=-nbx, index=level)
            ng = -(-rows // GROUP)
            assert flat.numel() == ng * GROUP * nby * nbx * bh * bw
            assert torch.equal(untile(flat, rows, h, w, -nbx, level)[:, 0], lv)
            sz = nby * nbx * bh * bw
            for r, y, x in [(rows - 1, h - 1, w - 1), (0, 0, 0), (rows // 2, h // 2, w - 1)]:
                off = ((r // GROUP) * GROUP * sz + (((y // bh) * nbx + x // bw) * GROUP + r % GROUP) * bh * bw
                       + (y % bh) * bw + x % bw)
                assert flat[off] == lv[r, y, x]


def test_split_build_arguments(ea):
    from eraft_amd import _lib
    L = _lib.lib()
    n = ctypes.c_int64()
    # exponents (2 x B x 4800 ints, 256-B aligned) + 8-KB f16 hi/lo panels per (tile, 16-deep chunk):
    # 38 query tiles and 38 target tiles (35 8x16 blocks + 3 4x32 band blocks) at 60 x 80
    assert L.ecorr_build_split_workspace_size(16, 256, 60, 80, 4800, ctypes.byref(n)) == 0
    assert n.value == 2 * 16 * 4800 * 4 + 2 * 16 * 38 * 16 * 8192
    # query slab of 20 rows x 160 of a 92 x 160 map: 25 query tiles; 11 x 10 + 5 band target tiles
    assert L.ecorr_build_split_workspace_size(4, 256, 92, 160, 3200, ctypes.byref(n)) == 0
    ex = (4 * 3200 * 4 + 4 * 92 * 160 * 4 + 255) // 256 * 256
    assert n.value == ex + 4 * 25 * 16 * 8192 + 4 * 115 * 16 * 8192
    assert L.ecorr_build_split_workspace_size(0, 256, 60, 80, 4800, ctypes.byref(n)) == _lib.ECORR_EINVAL
    assert L.ecorr_build_split_workspace_size(1, 256, 60, 80, 4801, ctypes.byref(n)) == _lib.ECORR_EINVAL
    assert L.ecorr_build_split(8, 8, 1, 256, 8, 8, 64, 4, 8, None, None) == _lib.ECORR_EINVAL
    with pytest.raises(ValueError):
        _lib.set_build_mode("bf16")


def test_pmc_source_digest_matches_library_digest(ea):
    """bench.py ties roofline.traffic to the kernel sources a PMC summary measured; the summary
    tool and the package must hash the same files the same way."""
    path = os.path.join(ROOT, "tools", "pmc_summary.py")
    src = open(path).read()
    ns = {"__file__": path}
    exec(compile(src.split("root = sys.argv[1]")[0], path, "exec"), ns)
    assert ns["source_digest"]() == ea._lib.source_digest()


def test_pmc_traffic_is_shape_keyed(tmp_path):
    """bench.py reports roofline.traffic only from a PMC record of its own launch shape and its own
    kernel sources; another config's record is refused (the C5 line carried C2's bytes)."""
    import json
    import bench
    import eraft_amd
    dig = eraft_amd._lib.source_digest()
    rec = {"kernels": {"build_split_kernel<true, 16>": {"hbm_bytes": 2.29e9, "read_correction": "x2"}}}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"source": "t", "source_digest": dig, "shapes": {"B16_D256_q4800_60x80": rec}}))
    got, src = bench.pmc_traffic("build_split_kernel", "B16_D256_q4800_60x80", str(p))
    assert got == 2.29e9 and "B16_D256_q4800_60x80" in src
    got, src = bench.pmc_traffic("build_split_kernel", "B4_D256_q14720_92x160", str(p))
    assert got is None and src.startswith("refused: shape")
    p.write_text(json.dumps({"source": "t", "source_digest": "0" * 16, "shapes": {"B16_D256_q4800_60x80": rec}}))
    got, src = bench.pmc_traffic("build_split_kernel", "B16_D256_q4800_60x80", str(p))
    assert got is None and src.startswith("refused")
    assert bench.shape_key(4, 256, 92, 160, 92 * 160) == "B4_D256_q14720_92x160"
