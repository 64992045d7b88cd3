"""eraft_amd -- MI355X-native (gfx950) E-RAFT correlation hot path.

Drop-in for wzygzlm/E-RAFT's model/corr.py and the model/utils.py hot-path helpers:

    from eraft_amd import CorrBlock, bilinear_sampler, coords_grid

The package lives in the hyphenated directory e-raft_amd/; the root module eraft_amd.py makes it
importable as `eraft_amd`.  Kernels: e-raft_amd/csrc (HIP, C ABI include/ecorr.h).
"""
from .corr import CorrBlock
from .utils import bilinear_sampler, coords_grid
from .image_utils import forward_interpolate_pytorch, grid_sample_values
from .flow import flow_16bit_to_float, flow_to_png16, upsample_flow
from .voxel import EventSequenceToVoxelGrid_Pytorch, VoxelGrid
from ._lib import LIB_PATH, lib

__all__ = ["CorrBlock", "bilinear_sampler", "coords_grid", "forward_interpolate_pytorch", "grid_sample_values",
           "upsample_flow", "flow_to_png16", "flow_16bit_to_float",
           "VoxelGrid", "EventSequenceToVoxelGrid_Pytorch", "LIB_PATH", "lib"]
