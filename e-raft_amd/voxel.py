"""Event -> voxel grid on MI355X, the input side of E-RAFT.

    VoxelGrid((C, H, W), normalize=True).convert({'p', 't', 'x', 'y'})     # utils/dsec_utils.py:19-64
    EventSequenceToVoxelGrid_Pytorch(num_bins, normalize=True)(sequence)  # utils/transformers.py:18-126

Same classes, arguments and results as the reference; the accumulated grid is bit-exact with the
reference's (single-threaded, main.py:2-5) serial fold and the nonzero normalization agrees within
an ulp or two (voxel.hip).  No CPU path: the DSEC events must be fp32 HIP tensors; the MVSEC
sequence's float64 features are copied to the HIP device like the reference's gpu=True mode.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def _workspace(dsec, n, C, H, W, device):
    nbytes = ctypes.c_int64()
    _lib.check(_lib.lib().ecorr_voxel_workspace_size(int(dsec), n, C, H, W, ctypes.byref(nbytes)),
               "voxel workspace")
    return torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=device)


class VoxelGrid:
    """dsec_utils.py:19-64: trilinear (x, y, t) voting of DSEC events into [C, H, W]."""

    def __init__(self, input_size: tuple, normalize: bool):
        assert len(input_size) == 3
        self.nb_channels, self.height, self.width = (int(v) for v in input_size)
        self.normalize = normalize

    def convert(self, events):
        C, H, W = self.nb_channels, self.height, self.width
        ts = [events[k] for k in ("p", "t", "x", "y")]
        for name, t in zip("ptxy", ts):
            if not isinstance(t, torch.Tensor) or t.device.type != "cuda" or t.dtype != torch.float32:
                raise RuntimeError(f"events['{name}'] must be a float32 HIP tensor (no CPU path)")
        n = ts[0].numel()
        if any(t.numel() != n for t in ts):
            raise RuntimeError("events p, t, x, y differ in length")
        if n == 0:   # the reference indexes t_norm[0]
            raise IndexError("index 0 is out of bounds for dimension 0 with size 0")
        p, t, x, y = (v.reshape(-1).contiguous() for v in ts)
        dev = p.device
        with torch.no_grad(), torch.cuda.device(dev):
            voxel = torch.empty((C, H, W), dtype=torch.float32, device=dev)
            ws = _workspace(True, n, C, H, W, dev)
            _lib.check(_lib.lib().ecorr_voxel_grid_dsec(
                p.data_ptr(), t.data_ptr(), x.data_ptr(), y.data_ptr(), n, C, H, W, int(bool(self.normalize)),
                voxel.data_ptr(), ws.data_ptr(), _lib.stream_of(p)), "VoxelGrid.convert")
        return voxel


class EventSequenceToVoxelGrid_Pytorch:
    """transformers.py:18-126: temporal-bilinear voting of [N, 4] (t, x, y, p) float64 events."""

    def __init__(self, num_bins, gpu=True, gpu_nr=0, normalize=True, forkserver=True):
        self.num_bins = num_bins
        self.normalize = normalize
        if not torch.cuda.is_available():
            raise RuntimeError("EventSequenceToVoxelGrid_Pytorch: no HIP device (eraft_amd has no CPU path)")
        self.device = torch.device("cuda", gpu_nr)   # gpu=False is served on the device too

    def __call__(self, event_sequence):
        events = event_sequence.features
        width, height = event_sequence.image_width, event_sequence.image_height
        assert events.shape[1] == 4
        assert self.num_bins > 0
        assert width > 0
        assert height > 0
        if isinstance(events, np.ndarray):
            ev = torch.from_numpy(np.ascontiguousarray(events, dtype=np.float64)).to(self.device)
        else:
            ev = events.to(self.device, torch.float64).contiguous()
        n = ev.shape[0]
        if n == 0:
            raise IndexError("index -1 is out of bounds for dimension 0 with size 0")
        with torch.no_grad(), torch.cuda.device(self.device):
            voxel = torch.empty((self.num_bins, height, width), dtype=torch.float32, device=self.device)
            bad = torch.zeros((1,), dtype=torch.int32, device=self.device)
            ws = _workspace(False, n, self.num_bins, height, width, self.device)
            _lib.check(_lib.lib().ecorr_voxel_grid_mvsec(
                ev.data_ptr(), n, self.num_bins, height, width, int(bool(self.normalize)), voxel.data_ptr(),
                bad.data_ptr(), ws.data_ptr(), _lib.stream_of(ev)), "EventSequenceToVoxelGrid_Pytorch")
            if int(bad.item()):
                raise IndexError("index out of range in self")   # the reference's index_add_
        return voxel
