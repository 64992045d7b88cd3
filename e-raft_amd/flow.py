"""Flow output side on MI355X: convex upsampling and the DSEC 16-bit PNG codec.

    up = upsample_flow(flow, mask)           # ERAFT.upsample_flow, model/eraft.py:74-85
    png = flow_to_png16(flow)                # the array visualize_flow_submission writes,
                                             #   utils/visualization.py:75-93
    flow, valid = flow_16bit_to_float(png)   # utils/dsec_utils.py:66-83

One HIP launch each (upsample.hip).  upsample_flow agrees with the reference within a few ulp
(device expf); the codec is bit-exact.  No CPU path: inputs must be HIP tensors.
"""
import torch

from . import _lib


def _require_device(name, t, dtype):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} is on {t.device}: eraft_amd runs only on HIP devices (no CPU path)")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype} (got {t.dtype})")


def upsample_flow(flow, mask):
    """eraft.py:74-85: flow [N, 2, H, W], mask [N, 576, H, W] -> [N, 2, 8H, 8W]."""
    _require_device("flow", flow, torch.float32)
    _require_device("mask", mask, torch.float32)
    if flow.dim() != 4 or flow.shape[1] != 2:
        raise RuntimeError(f"flow must be [N, 2, H, W], got {tuple(flow.shape)}")
    N, _, H, W = flow.shape
    if mask.numel() != N * 576 * H * W:   # the reference's mask.view(N, 1, 9, 8, 8, H, W)
        raise RuntimeError(f"shape '[{N}, 1, 9, 8, 8, {H}, {W}]' is invalid for input of size {mask.numel()}")
    flow, mask = flow.contiguous(), mask.contiguous()
    with torch.cuda.device(flow.device):
        out = torch.empty((N, 2, 8 * H, 8 * W), dtype=torch.float32, device=flow.device)
        _lib.check(_lib.lib().ecorr_upsample_flow(flow.data_ptr(), mask.data_ptr(), N, H, W, out.data_ptr(),
                                                  _lib.stream_of(flow)), "upsample_flow")
    return out


def flow_to_png16(flow):
    """visualization.py:81-84: flow [2, h, w] (or [B, 2, h, w]) -> uint16 [h, w, 3] ([B, h, w, 3]):
    rint(flow * 128 + 2^15) cast like numpy's astype(uint16), channel 2 = 0."""
    _require_device("flow", flow, torch.float32)
    single = flow.dim() == 3
    f = flow.unsqueeze(0) if single else flow
    if f.dim() != 4 or f.shape[1] != 2:
        raise RuntimeError(f"flow must be [2, h, w] or [B, 2, h, w], got {tuple(flow.shape)}")
    f = f.contiguous()
    B, _, h, w = f.shape
    with torch.cuda.device(f.device):
        out = torch.empty((B, h, w, 3), dtype=torch.uint16, device=f.device)
        _lib.check(_lib.lib().ecorr_flow_to_png16(f.data_ptr(), B, h, w, out.data_ptr(), _lib.stream_of(f)),
                   "flow_to_png16")
    return out[0] if single else out


def flow_16bit_to_float(flow_16bit):
    """dsec_utils.py:66-83: uint16 [h, w, 3] -> (flow [h, w, 2] float32, valid [h, w] bool).
    The reference returns float64; every value (v - 2^15) / 128 is exact in float32.  Raises
    AssertionError where the reference asserts (dtype, shape, channel 2 outside {0, 1})."""
    if not isinstance(flow_16bit, torch.Tensor):
        raise TypeError("flow_16bit must be a torch.Tensor")
    assert flow_16bit.dtype == torch.uint16
    assert flow_16bit.dim() == 3
    h, w, c = flow_16bit.shape
    assert c == 3
    _require_device("flow_16bit", flow_16bit, torch.uint16)
    src = flow_16bit.contiguous()
    dev = src.device
    with torch.cuda.device(dev):
        flow = torch.empty((h, w, 2), dtype=torch.float32, device=dev)
        valid = torch.empty((h, w), dtype=torch.bool, device=dev)
        bad = torch.zeros((1,), dtype=torch.int32, device=dev)
        _lib.check(_lib.lib().ecorr_png16_to_flow(src.data_ptr(), 1, h, w, flow.data_ptr(), valid.data_ptr(),
                                                  bad.data_ptr(), _lib.stream_of(src)), "flow_16bit_to_float")
        assert int(bad.item()) == 0, "flow_16bit: invalid pixels must have channel 2 == 0"
    return flow, valid
