"""GPU parity of the warm-start splat (splat.hip) through the C ABI:
bit-exact against the reference's goldens and against the serial CPU oracle at the configs'
sizes; deterministic run to run."""
import os

import numpy as np
import pytest
import torch

import oracle
import prng

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ea():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


@pytest.fixture(scope="module")
def splat():
    return np.load(os.path.join(GOLD, "next_splat.npz"))


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_forward_interpolate_goldens(ea, splat):
    names = sorted(k.split("/")[0] for k in splat.files if k.startswith("fi_") and k.endswith("/flow"))
    for k in names:
        got = ea.forward_interpolate_pytorch(_dev(splat[f"{k}/flow"])).cpu().numpy()
        assert oracle.same_bits(got, splat[f"{k}/out"]), k


def test_grid_sample_values_goldens(ea, splat):
    names = sorted(k.split("/")[0] for k in splat.files if k.startswith("gsv_") and k.endswith("/input"))
    for k in names:
        h, w = (int(v) for v in splat[f"{k}/hw"])
        values, valid = ea.grid_sample_values(_dev(splat[f"{k}/input"]), h, w)
        assert valid.dtype == torch.bool and tuple(values.shape) == (1, h, w)
        assert oracle.same_bits(values.cpu().numpy(), splat[f"{k}/values"]), k
        assert np.array_equal(valid.cpu().numpy(), splat[f"{k}/valid"]), k


@pytest.mark.parametrize("B,h,w,sigma", [
    (16, 60, 80, 1.5),     # DSEC warm start (configs[1])
    (64, 32, 32, 1.5),     # MVSEC (configs[2])
    (4, 92, 160, 3.0),     # 1280x720 (configs[4])
    (1, 130, 140, 4.0),    # > 16384 targets: counts in the workspace instead of LDS
    (1, 264, 300, 3.0),    # > 65536 points: the one-workgroup-per-item kernel and its workspace
    (2, 7, 300, 40.0),     # mostly out of the image
])
def test_forward_interpolate_vs_oracle(ea, B, h, w, sigma):
    flow = prng.normal(200 + h, (B, 2, h, w), sigma)
    got = ea.forward_interpolate_pytorch(_dev(flow))
    again = ea.forward_interpolate_pytorch(_dev(flow))
    ref = oracle.forward_interpolate(flow)
    assert oracle.same_bits(got.cpu().numpy(), ref)
    assert torch.equal(got, again)   # deterministic (no float atomics)


def test_collisions_vs_oracle(ea):
    # every pixel of a 60x80 map lands within a few pixels of one point: buckets of ~1000 keys
    h, w = 60, 80
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    flow = np.stack([(40.25 - xx) * 0.99, (30.5 - yy) * 0.99])[None].astype(np.float32)
    flow = np.ascontiguousarray(np.repeat(flow, 3, axis=0))
    got = ea.forward_interpolate_pytorch(_dev(flow)).cpu().numpy()
    assert oracle.same_bits(got, oracle.forward_interpolate(flow))


def test_one_target_holds_everything(ea):
    """Every pixel moves exactly onto one integer target: its 4 passes all land there (floor = ceil),
    19,200 contributions in one bucket -- more than a band's list holds, so the banded kernel folds
    that target by walking the contributions in (pass, point) order."""
    h, w = 60, 80
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    flow = np.stack([40.0 - xx, 30.0 - yy])[None].astype(np.float32)
    flow = np.ascontiguousarray(np.repeat(flow, 2, axis=0))
    got = ea.forward_interpolate_pytorch(_dev(flow)).cpu().numpy()
    assert oracle.same_bits(got, oracle.forward_interpolate(flow))


def test_grid_sample_values_many_points_vs_oracle(ea):
    """> 65536 points: the workspace path (banded kernel only up to 65536 points per item)."""
    n, h, w = 70_000, 120, 150
    pts = prng.uniform(7, (3, n), -2.0, 1.0).astype(np.float32)
    pts[0] = (pts[0] + 2.0) / 3.0 * (w + 1) - 1.0
    pts[1] = (pts[1] + 2.0) / 3.0 * (h + 1) - 1.0
    values, valid = ea.grid_sample_values(_dev(pts), h, w)
    ref_v, ref_m = oracle.grid_sample_values(pts, h, w)
    assert oracle.same_bits(values.cpu().numpy(), ref_v)
    assert np.array_equal(valid.cpu().numpy(), ref_m)


def test_splat_rejects_cpu_and_bad_shapes(ea):
    with pytest.raises(RuntimeError):
        ea.forward_interpolate_pytorch(torch.zeros(1, 2, 4, 4))
    with pytest.raises(RuntimeError):
        ea.forward_interpolate_pytorch(torch.zeros(1, 3, 4, 4, device="cuda"))
    with pytest.raises(RuntimeError):
        ea.grid_sample_values(torch.zeros(2, 5, device="cuda"), 4, 4)


def test_batch_past_grid_y_limit(ea):
    """the banded splat once put the batch on gridDim.y (limit 65535); with a linear block
    index a batch of 65,600 small maps runs, and every item equals the same item splatted alone."""
    B, h, w = 65600, 3, 4
    g = torch.Generator(device="cuda").manual_seed(11)
    flow = (torch.randn((B, 2, h, w), generator=g, device="cuda") * 1.5).contiguous()
    out = ea.forward_interpolate_pytorch(flow)
    for i in (0, 1, 65534, 65535, 65536, B - 1):
        assert torch.equal(out[i:i + 1], ea.forward_interpolate_pytorch(flow[i:i + 1].contiguous())), i
