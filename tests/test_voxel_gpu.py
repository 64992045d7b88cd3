"""GPU parity of the event -> voxel grid (voxel.hip) through the C ABI: the
accumulated grid bit-exact with the reference's serial fold (goldens, and the oracle at DSEC full
resolution with 1M events); the normalized grid within NORM_TOL (reduction order only)."""
import os

import numpy as np
import pytest
import torch

import oracle
import prng
from voxel_cases import DSEC_VOXEL, MVSEC_VOXEL, dsec_case, mvsec_case

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NORM_TOL = 1e-6   # rtol and atol on the normalized grid


@pytest.fixture(scope="module")
def ea():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


@pytest.fixture(scope="module")
def voxz():
    return np.load(os.path.join(GOLD, "next_voxel.npz"))


class _Seq:
    pass


def _dsec(ea, p, t, x, y, C, H, W, norm):
    ev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in zip("ptxy", (p, t, x, y))}
    return ea.VoxelGrid((C, H, W), normalize=norm).convert(ev).cpu().numpy()


def _mvsec(ea, ev, C, H, W, norm):
    s = _Seq()
    s.features, s.image_width, s.image_height = ev, W, H
    return ea.EventSequenceToVoxelGrid_Pytorch(C, gpu=True, normalize=norm)(s).cpu().numpy()


def test_voxel_dsec_goldens(ea, voxz):
    for k, (n, C, H, W, seed) in DSEC_VOXEL.items():
        p, t, x, y = dsec_case(k, n, H, W, seed)
        assert oracle.same_bits(_dsec(ea, p, t, x, y, C, H, W, False), voxz[f"{k}/norm0"]), k
        np.testing.assert_allclose(_dsec(ea, p, t, x, y, C, H, W, True), voxz[f"{k}/norm1"],
                                   rtol=NORM_TOL, atol=NORM_TOL, err_msg=k)


def test_voxel_mvsec_goldens(ea, voxz):
    for k, (n, C, H, W, seed) in MVSEC_VOXEL.items():
        ev = mvsec_case(k, n, H, W, seed)
        if f"{k}/raises" in voxz.files:
            with pytest.raises(IndexError):
                _mvsec(ea, ev, C, H, W, True)
            continue
        assert oracle.same_bits(_mvsec(ea, ev, C, H, W, False), voxz[f"{k}/norm0"]), k
        np.testing.assert_allclose(_mvsec(ea, ev, C, H, W, True), voxz[f"{k}/norm1"],
                                   rtol=NORM_TOL, atol=NORM_TOL, err_msg=k)


def test_voxel_dsec_full_res_vs_oracle(ea):
    # DSEC 15 x 480 x 640 with 1M events: bit-exact accumulation, deterministic run to run
    n, C, H, W = 1_000_000, 15, 480, 640
    p, t, x, y = prng.dsec_events(700, n, H, W)
    g = _dsec(ea, p, t, x, y, C, H, W, False)
    assert oracle.same_bits(g, oracle.voxel_dsec(p, t, x, y, C, H, W, False))
    g1 = _dsec(ea, p, t, x, y, C, H, W, True)
    np.testing.assert_allclose(g1, oracle.voxel_dsec(p, t, x, y, C, H, W, True), rtol=NORM_TOL, atol=NORM_TOL)
    assert np.array_equal(g1, _dsec(ea, p, t, x, y, C, H, W, True))


def test_voxel_mvsec_full_res_vs_oracle(ea):
    n, C, H, W = 300_000, 15, 260, 346
    ev = prng.mvsec_events(710, n, H, W)
    g = _mvsec(ea, ev, C, H, W, False)
    ref, bad = oracle.voxel_mvsec(ev, C, H, W, False)
    assert not bad and oracle.same_bits(g, ref)


@pytest.mark.parametrize("case", ["hot_pixel", "dense_ragged", "sparse_ragged", "unsorted_t", "c23_run_table_full",
                                  "c24_key_range_fallback"])
def test_voxel_dsec_tiled_paths_vs_oracle(ea, case):
    """The tiled DSEC path (round 6): 4 x 16 cell tiles, each reading its window (its base cells and
    the +1 halo, every time bin) from one contiguous bucket -- in LDS, or past VB_CAP = 512 events
    where it lies in HBM with its run order in the global arena.  hot_pixel: 60% of the events on one
    base cell (~12,000 in one window: the arena, runs of thousands ranked by event index);
    dense_ragged: every window past the cap (~1,800 events each), tiles cut by H % 4 and W % 16;
    sparse_ragged: the LDS path on partial tiles; unsorted_t: timestamps not in order (a bucket then
    interleaves bins' events arbitrarily); C = 23: the run table full (2,040 of 2,048), C = 24: the
    key-range pipeline instead.  Accumulated grid bit-exact with the serial fold, normalized within
    NORM_TOL."""
    if case == "hot_pixel":
        n, C, H, W = 20_000, 3, 16, 64
        p, t, x, y = prng.dsec_events(730, n, H, W)
        hot = prng.uniform(731, (n,)) < 0.6
        x[hot] = np.float32(10.3)
        y[hot] = np.float32(5.7)
    elif case == "dense_ragged":
        n, C, H, W = 60_000, 4, 21, 130
        p, t, x, y = prng.dsec_events(740, n, H, W)
    elif case == "sparse_ragged":
        n, C, H, W = 3_000, 5, 21, 70
        p, t, x, y = prng.dsec_events(750, n, H, W)
    elif case == "unsorted_t":
        n, C, H, W = 8_000, 4, 30, 90
        p, t, x, y = prng.dsec_events(760, n, H, W)
        t = t[np.argsort(prng.uniform(761, (n,)))].copy()   # a permutation: t[0], t[-1] arbitrary
    else:   # (C + 1) * 85 runs per window: 2,040 at C = 23 (the LDS table's last fit), C = 24 the fallback
        n, H, W = 20_000, 13, 37
        C = 23 if case == "c23_run_table_full" else 24
        p, t, x, y = prng.dsec_events(770 + C, n, H, W)
    g = _dsec(ea, p, t, x, y, C, H, W, False)
    assert oracle.same_bits(g, oracle.voxel_dsec(p, t, x, y, C, H, W, False)), case
    np.testing.assert_allclose(_dsec(ea, p, t, x, y, C, H, W, True), oracle.voxel_dsec(p, t, x, y, C, H, W, True),
                               rtol=NORM_TOL, atol=NORM_TOL, err_msg=case)


def test_voxel_normalize_unaligned_output(ea):
    """norm_apply's 16-byte path needs a 16-byte-aligned grid: an output 4 bytes into a buffer takes
    the scalar kernel, and C * H * W = 105 (n % 4 = 1) exercises the vector path's tail; both equal
    the aligned run bit for bit."""
    import ctypes
    from eraft_amd import _lib, voxel
    n, C, H, W = 2_000, 3, 5, 7
    p, t, x, y = (torch.from_numpy(v).cuda() for v in prng.dsec_events(770, n, H, W))
    ref = ea.VoxelGrid((C, H, W), normalize=True).convert({"p": p, "t": t, "x": x, "y": y})
    buf = torch.full((C * H * W + 1,), float("nan"), device="cuda")
    out = buf[1:]
    assert out.data_ptr() % 16 == 4
    ws = voxel._workspace(True, n, C, H, W, p.device)
    _lib.check(_lib.lib().ecorr_voxel_grid_dsec(p.data_ptr(), t.data_ptr(), x.data_ptr(), y.data_ptr(), n, C, H, W,
                                                1, out.data_ptr(), ws.data_ptr(), _lib.stream_of(p)), "voxel")
    torch.cuda.synchronize()
    assert torch.equal(out.view(C, H, W), ref)
    assert (ref != 0).any()


def test_voxel_rejects_cpu_events(ea):
    p, t, x, y = prng.dsec_events(720, 10, 4, 4)
    with pytest.raises(RuntimeError):
        ea.VoxelGrid((2, 4, 4), True).convert({k: torch.from_numpy(v) for k, v in zip("ptxy", (p, t, x, y))})
