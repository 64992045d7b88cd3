"""Warm-start splat on MI355X (mirrors /root/reference/utils/image_utils.py:10-83).

    flow_init = forward_interpolate_pytorch(flow_low_res)        # image_utils.py:50 (test.py:199)
    values, valid = grid_sample_values(input, height, width)     # image_utils.py:10

Same signatures and results as the reference -- bit-exact with its CPU put_(accumulate=True),
which folds each target's contributions serially (the reference on a GPU uses float atomics and
is not even reproducible run to run).  The whole batch is one kernel launch (splat.hip) instead
of the reference's per-sample Python loop (:78-80), so warm start works at any batch size (the
reference restricts it to B = 1, test.py:144).  No CPU path: inputs must be fp32 HIP tensors.
"""
import ctypes

import torch

from . import _lib


def _require_device_f32(name, t):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} is on {t.device}: eraft_amd runs only on HIP devices (no CPU path)")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")


_WS_BYTES = {}


def _workspace(B, n, h, w, device):
    """The splat's scratch (ecorr_splat_workspace_size), or None when the shape needs none (the banded
    kernel: n <= 65536 points per item); sizes are cached per shape."""
    key = (B, n, h, w)
    nb = _WS_BYTES.get(key)
    if nb is None:
        nbytes = ctypes.c_int64()
        _lib.check(_lib.lib().ecorr_splat_workspace_size(B, n, h, w, ctypes.byref(nbytes)), "splat workspace")
        nb = _WS_BYTES[key] = nbytes.value
    return torch.empty(nb, dtype=torch.uint8, device=device) if nb > 0 else None


def grid_sample_values(input, height, width):
    """image_utils.py:10-47: input [3, N] rows (x, y, z) -> (values [1, H, W], valid_mask [1, H, W] bool)."""
    _require_device_f32("input", input)
    if input.dim() != 2 or input.shape[0] != 3:
        raise RuntimeError(f"input must be [3, N] (x, y, z), got {tuple(input.shape)}")
    pts = input.contiguous()
    n = pts.shape[1]
    dev = pts.device
    with torch.cuda.device(dev):
        values = torch.empty((1, height, width), dtype=torch.float32, device=dev)
        valid = torch.empty((1, height, width), dtype=torch.bool, device=dev)
        ws = _workspace(1, n, height, width, dev)
        _lib.check(_lib.lib().ecorr_grid_sample_values(
            pts.data_ptr() if n else None, n, height, width, values.data_ptr(), valid.data_ptr(),
            None if ws is None else ws.data_ptr(), _lib.stream_of(pts)), "grid_sample_values")
    return values, valid


def forward_interpolate_pytorch(flow_in):
    """image_utils.py:50-83: flow [B, 2, H, W] (or [2, H, W]) -> forward-splatted flow [B, 2, H, W]."""
    _require_device_f32("flow_in", flow_in)
    flow = flow_in.unsqueeze(0) if flow_in.dim() < 4 else flow_in
    if flow.dim() != 4 or flow.shape[1] != 2:
        raise RuntimeError(f"flow must be [B, 2, H, W], got {tuple(flow_in.shape)}")
    flow = flow.contiguous()
    b, _, h, w = flow.shape
    dev = flow.device
    with torch.cuda.device(dev):
        out = torch.empty((b, 2, h, w), dtype=torch.float32, device=dev)
        if b == 0:
            return out
        ws = _workspace(b, h * w, h, w, dev)
        _lib.check(_lib.lib().ecorr_forward_interpolate(
            flow.data_ptr(), b, h, w, out.data_ptr(), None if ws is None else ws.data_ptr(), _lib.stream_of(flow)),
            "forward_interpolate")
    return out
