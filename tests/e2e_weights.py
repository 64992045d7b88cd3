"""Deterministic 'random-init' ERAFT weights (test infrastructure).

The reference checkpoints (dsec.tar, mvsec_*.tar) are download-only and absent, so end-to-end
parity runs both networks on the same PRNG weights: every state_dict entry is drawn from
tests/prng.py with a seed derived from its key, so the golden capture (reference ERAFT) and the
GPU test (e-raft_amd's ERAFT counterpart, same keys) load bit-identical tensors.
"""
import zlib

import numpy as np
import torch

import prng


def key_seed(name: str) -> int:
    return zlib.crc32(name.encode()) & 0x7FFFFFFF


def make_state_dict(template):
    sd = {}
    for name, t in template.items():
        shape = tuple(t.shape)
        s = key_seed(name)
        if name.endswith("num_batches_tracked"):
            sd[name] = torch.zeros_like(t)
            continue
        if name.endswith("running_var"):
            v = prng.uniform(s, shape, 0.5, 1.5)
        elif name.endswith("running_mean"):
            v = prng.normal(s, shape, 0.1)
        elif name.endswith("weight") and len(shape) == 4:      # conv: kaiming-normal, fan_in
            fan_in = int(np.prod(shape[1:]))
            v = prng.normal(s, shape, float(np.sqrt(2.0 / fan_in)))
        elif name.endswith("weight"):                          # norm affine scale
            v = (1.0 + prng.normal(s, shape, 0.1)).astype(np.float32)
        else:                                                  # biases
            v = prng.normal(s, shape, 0.01)
        sd[name] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)).to(t.dtype)
    return sd
