"""Deterministic 'random-init' ERAFT weights (test infrastructure).

The reference checkpoints (dsec.tar, mvsec_*.tar) are download-only and absent, so end-to-end
parity runs both networks on the same PRNG weights: every state_dict entry is drawn from
tests/prng.py with a seed derived from its key, so the golden capture (reference ERAFT) and the
GPU test (e-raft_amd's ERAFT counterpart, same keys) load bit-identical tensors.

Scales follow the reference's own initialisation, i.e. what ERAFT(config) itself produces:
encoder convs kaiming-normal fan_out/relu (extractor.py:133-136), every other conv PyTorch's
default (kaiming-uniform a=sqrt(5): std 1/sqrt(3 fan_in)), biases the default
U(+-1/sqrt(fan_in)) std; norm layers near (1, 0) with small perturbations and valid running stats.
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
        elif name.endswith("weight") and len(shape) == 4:      # conv weights
            encoder = name.startswith(("fnet.", "cnet."))
            fan_in = int(np.prod(shape[1:]))
            fan_out = shape[0] * int(np.prod(shape[2:]))
            std = np.sqrt(2.0 / fan_out) if encoder else 1.0 / np.sqrt(3.0 * fan_in)
            v = prng.normal(s, shape, float(std))
        elif name.endswith("weight"):                          # norm affine scale
            v = (1.0 + prng.normal(s, shape, 0.1)).astype(np.float32)
        elif name.endswith("bias") and name[:-len("bias")] + "weight" in template and \
                len(template[name[:-len("bias")] + "weight"].shape) == 4:   # conv bias
            w = template[name[:-len("bias")] + "weight"]
            fan_in = int(np.prod(tuple(w.shape)[1:]))
            v = prng.normal(s, shape, float(1.0 / np.sqrt(3.0 * fan_in)))
        else:                                                  # norm biases
            v = prng.normal(s, shape, 0.1)
        sd[name] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)).to(t.dtype)
    return sd
