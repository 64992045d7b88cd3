#!/usr/bin/env python3
"""Capture golden vectors for the SURVEY §8f "next" rows from the imported reference.

Run ONLY in the build container (the reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_next.py

Like make_golden.py: the reference (/root/reference, wzygzlm/E-RAFT) is imported read-only and run
on torch-CPU; inputs are drawn from tests/prng.py and stored alongside the reference's outputs.

  next_splat.npz    utils/image_utils.py forward_interpolate_pytorch (:50-83) on several flow
                    fields (sub-pixel, large/out-of-image, converging = many collisions, integer =
                    floor == ceil, NaN/inf, 3-D input) and grid_sample_values (:10-47) on scattered
                    points incl. the empty set.
  next_flow.npz     model/eraft.py ERAFT.upsample_flow (:74-85) on PRNG flows/masks (mask scales
                    0.25 .. 30: flat to one-hot softmax); the DSEC PNG codec: the submission
                    array of utils/visualization.py:81-84 (that module is not importable here --
                    its loader import needs h5py -- so its three numpy lines are evaluated as
                    written) and utils/dsec_utils.py flow_16bit_to_float (:66-83, imported),
                    incl. out-of-range / NaN / tie values and the assertion case.
  next_voxel.npz    utils/dsec_utils.py VoxelGrid.convert (:26-64) and utils/transformers.py
                    EventSequenceToVoxelGrid_Pytorch (:36-126) on prng.dsec_events /
                    prng.mvsec_events (seeds stored), normalize off and on, with torch pinned to
                    one thread as main.py:2-5 does; edge cases: constant timestamps, NaN
                    coordinates, one hot pixel, an out-of-grid MVSEC index (raises).
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (prng)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import prng  # noqa: E402
from voxel_cases import DSEC_VOXEL, MVSEC_VOXEL, dsec_case, mvsec_case  # noqa: E402
from model.eraft import ERAFT  # noqa: E402  (reference)
from utils.dsec_utils import VoxelGrid, flow_16bit_to_float  # noqa: E402  (reference)
from utils.transformers import EventSequenceToVoxelGrid_Pytorch  # noqa: E402  (reference)
from utils.image_utils import forward_interpolate_pytorch, grid_sample_values  # noqa: E402  (reference)

torch.set_num_threads(8)


def splat_cases():
    cases = {}
    cases["fi_dsec_s3"] = prng.normal(100, (2, 2, 60, 80), 3.0)
    cases["fi_s30"] = prng.normal(101, (1, 2, 24, 32), 30.0)
    h, w = 36, 44
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    conv = np.stack([(21.3 - xx) * 0.93, (17.6 - yy) * 0.93])[None]
    cases["fi_converge"] = (conv + prng.normal(102, (1, 2, h, w), 0.05)).astype(np.float32)
    cases["fi_int"] = np.round(prng.normal(103, (2, 2, 20, 28), 2.0)).astype(np.float32)
    f = prng.normal(104, (1, 2, 16, 24), 2.0)
    f[0, 0, 3, 5] = np.nan
    f[0, 1, 7, 9] = np.inf
    f[0, 0, 10, 2] = -np.inf
    f[0, 1, 0, 0] = 1e30
    cases["fi_special"] = f
    cases["fi_3d"] = prng.normal(105, (2, 12, 17), 1.5)   # [2, H, W] input -> [1, 2, H, W]
    cases["fi_mvsec"] = prng.normal(106, (4, 2, 32, 32), 1.5)
    out = {}
    for k, flow in cases.items():
        ref = forward_interpolate_pytorch(torch.from_numpy(flow.copy())).numpy()
        out[f"{k}/flow"] = flow
        out[f"{k}/out"] = ref
    # grid_sample_values on scattered points (n != h*w, some outside)
    for k, (n, h, w, seed) in {"gsv_scatter": (5000, 30, 40, 110), "gsv_dense": (20000, 9, 11, 111),
                               "gsv_empty": (0, 5, 7, 112)}.items():
        x = prng.uniform(seed, (n,), -3.0, w + 2.0)
        y = prng.uniform(seed + 1, (n,), -3.0, h + 2.0)
        z = prng.normal(seed + 2, (n,))
        inp = np.stack([x, y, z]).astype(np.float32).reshape(3, n)
        v, m = grid_sample_values(torch.from_numpy(inp.copy()), h, w)
        out[f"{k}/input"] = inp
        out[f"{k}/hw"] = np.array([h, w], dtype=np.int64)
        out[f"{k}/values"] = v.numpy()
        out[f"{k}/valid"] = m.numpy()
    return out


UPSAMPLE_CASES = {"up_small": (2, 6, 8, 1.0, 300), "up_dsec_crop": (1, 15, 20, 0.75, 310),
                  "up_onehot": (1, 4, 5, 30.0, 320), "up_flat": (1, 3, 7, 0.01, 330)}


def flow_cases():
    out = {}
    for k, (N, H, W, mscale, seed) in UPSAMPLE_CASES.items():
        flow = prng.normal(seed, (N, 2, H, W), 4.0)
        mask = prng.normal(seed + 1, (N, 576, H, W), mscale)
        ref = ERAFT.upsample_flow(None, torch.from_numpy(flow), torch.from_numpy(mask)).numpy()
        out[f"{k}/shape"] = np.array([N, H, W, seed], dtype=np.int64)
        out[f"{k}/mscale"] = np.array(mscale, dtype=np.float64)
        out[f"{k}/out"] = ref
    # encoder: flow [2, h, w] -> the uint16 [h, w, 3] array written to the submission PNG
    f = prng.normal(340, (2, 24, 32), 40.0)
    special = np.array([0.5 / 128, 1.5 / 128, -0.5 / 128, 2.5 / 128, 255.99, 256.0, -256.0, -300.0,
                        600.0, 1e9, -1e9, np.nan, np.inf, -np.inf, 1e-30, -0.0], dtype=np.float32)
    f.reshape(-1)[:special.size] = special
    for name, flow in {"enc_rand": f, "enc_small": prng.normal(341, (2, 5, 7), 3.0)}.items():
        _, h, w = flow.shape
        with np.errstate(invalid="ignore"):
            flow_map = np.rint(flow * 128 + 2 ** 15)                       # visualization.py:82
            flow_map = flow_map.astype(np.uint16).transpose(1, 2, 0)        # :83
        flow_map = np.concatenate((flow_map, np.zeros((h, w, 1), dtype=np.uint16)), axis=-1)   # :84
        out[f"{name}/flow"] = flow
        out[f"{name}/png"] = flow_map
    # decoder
    u = (prng.uniform(350, (40, 48, 3)) * 65536).astype(np.int64).clip(0, 65535).astype(np.uint16)
    u[..., 2] = (prng.uniform(351, (40, 48)) < 0.7).astype(np.uint16)
    fm, valid = flow_16bit_to_float(u.copy())
    out["dec/png"] = u
    out["dec/flow"] = fm
    out["dec/valid"] = valid
    bad = u.copy()
    bad[3, 4, 2] = 2
    try:
        flow_16bit_to_float(bad)
        raised = False
    except AssertionError:
        raised = True
    out["dec_bad/png"] = bad
    out["dec_bad/raises"] = np.array(raised)
    return out


class _Seq:
    pass


def voxel_cases():
    torch.set_num_threads(1)   # main.py:2-5
    out = {}
    for k, (n, C, H, W, seed) in DSEC_VOXEL.items():
        p, t, x, y = dsec_case(k, n, H, W, seed)
        out[f"{k}/shape"] = np.array([n, C, H, W, seed], dtype=np.int64)
        for norm in (0, 1):
            ev = {"p": torch.from_numpy(p.copy()), "t": torch.from_numpy(t.copy()),
                  "x": torch.from_numpy(x.copy()), "y": torch.from_numpy(y.copy())}
            out[f"{k}/norm{norm}"] = VoxelGrid((C, H, W), normalize=bool(norm)).convert(ev).numpy()
    for k, (n, C, H, W, seed) in MVSEC_VOXEL.items():
        ev = mvsec_case(k, n, H, W, seed)
        out[f"{k}/shape"] = np.array([n, C, H, W, seed], dtype=np.int64)
        for norm in (0, 1):
            s = _Seq()
            s.features, s.image_width, s.image_height = ev.copy(), W, H
            try:
                g = EventSequenceToVoxelGrid_Pytorch(C, gpu=False, normalize=bool(norm), forkserver=False)(s)
                out[f"{k}/norm{norm}"] = g.numpy()
            except (IndexError, RuntimeError):
                out[f"{k}/raises"] = np.array(True)
    torch.set_num_threads(8)
    return out


def main():
    np.savez_compressed(os.path.join(HERE, "next_splat.npz"), **splat_cases())
    print("wrote next_splat.npz")
    np.savez_compressed(os.path.join(HERE, "next_flow.npz"), **flow_cases())
    print("wrote next_flow.npz")
    np.savez_compressed(os.path.join(HERE, "next_voxel.npz"), **voxel_cases())
    print("wrote next_voxel.npz")


if __name__ == "__main__":
    main()
