"""Voxel-grid test cases shared by tests/golden/make_golden_next.py and the parity tests:
name -> (n events, C, H, W, seed) plus the edge-case edits each case applies to its events."""
import numpy as np

import prng

DSEC_VOXEL = {"vd_small": (3000, 5, 20, 30, 500), "vd_mid": (50000, 15, 48, 64, 510),
              "vd_const_t": (400, 3, 10, 12, 520), "vd_nan": (2000, 4, 16, 16, 530), "vd_hot": (5000, 5, 8, 8, 540)}
MVSEC_VOXEL = {"vm_small": (3000, 5, 26, 34, 600), "vm_mid": (50000, 15, 48, 64, 610),
               "vm_const_t": (300, 5, 6, 7, 620), "vm_hot": (4000, 15, 4, 5, 630), "vm_bad": (100, 5, 6, 7, 640)}


def dsec_case(k, n, H, W, seed):
    p, t, x, y = prng.dsec_events(seed, n, H, W)
    if k == "vd_const_t":
        t[:] = 5.0
    if k == "vd_nan":
        x[::97] = np.nan
        y[5::89] = np.inf
    if k == "vd_hot":
        x[:] = 3.25
        y[:] = 4.75
    return p, t, x, y


def mvsec_case(k, n, H, W, seed):
    ev = prng.mvsec_events(seed, n, H, W)
    if k == "vm_const_t":
        ev[:, 0] = 7.0
    if k == "vm_hot":
        ev[:, 1] = 2.0
        ev[:, 2] = 3.0
    if k == "vm_bad":
        ev[17, 1] = W * H * 99.0
    return ev
