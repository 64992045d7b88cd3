"""Hot-path helpers of /root/reference/model/utils.py, on gfx950 kernels.

bilinear_sampler(img, coords, mode='bilinear', mask=False)   utils.py:7-21
coords_grid(batch, ht, wd, device=None)                      utils.py:24-27
"""
import torch

from . import _lib
from .corr import _no_grad_inputs, _require_device_f32


def bilinear_sampler(img, coords, mode="bilinear", mask=False):
    """grid_sample(img, normalized(coords), align_corners=True, zeros padding) in pixel units.

    img [N, C, H, W], coords [N, Hg, Wg, 2] (x, y) -> [N, C, Hg, Wg]; with mask=True also the
    [N, Hg, Wg, 1] in-range mask.  Like the reference, `mode` is accepted and ignored (the
    reference never forwards it to grid_sample, utils.py:15).  Bit-exact with the reference CPU.
    """
    _require_device_f32("img", img)
    _require_device_f32("coords", coords)
    _no_grad_inputs(img, coords)
    if img.dim() != 4 or coords.dim() != 4 or coords.shape[-1] != 2 or coords.shape[0] != img.shape[0]:
        raise RuntimeError(f"bilinear_sampler: img {tuple(img.shape)} / coords {tuple(coords.shape)}")
    N, C, h, w = img.shape
    _, Hg, Wg, _ = coords.shape
    img = img.contiguous()
    coords = coords.contiguous()
    with torch.cuda.device(img.device):
        out = torch.empty((N, C, Hg, Wg), dtype=torch.float32, device=img.device)
        m = torch.empty((N, Hg, Wg, 1), dtype=torch.float32, device=img.device) if mask else None
        _lib.check(_lib.lib().ecorr_bilinear_sampler(
            img.data_ptr(), N, C, h, w, coords.data_ptr(), Hg, Wg, out.data_ptr(),
            m.data_ptr() if mask else None, _lib.stream_of(img)), "bilinear_sampler")
    return (out, m) if mask else out


def coords_grid(batch, ht, wd, device=None):
    """[batch, 2, ht, wd] grid, channel 0 = x (column), channel 1 = y (row).

    device=None returns a CPU tensor, as the reference does (its caller moves it, eraft.py:68);
    a HIP device builds it in place with the ecorr_coords_grid kernel.
    """
    if device is None or torch.device(device).type == "cpu":
        ys, xs = torch.meshgrid(torch.arange(ht), torch.arange(wd), indexing="ij")
        return torch.stack([xs, ys]).float()[None].repeat(batch, 1, 1, 1)
    device = torch.device(device)
    with torch.cuda.device(device):
        out = torch.empty((batch, 2, ht, wd), dtype=torch.float32, device=device)
        _lib.check(_lib.lib().ecorr_coords_grid(batch, ht, wd, out.data_ptr(), _lib.stream_of(out)),
                   "coords_grid")
    return out
