#!/usr/bin/env python3
"""Interleaved A/B of the CorrBlock build between the tree's libecorr.so and AB_ALT_LIB (another
build of the library, e.g. the previous round's: tools/r1_lab/libecorr_r1.so) in ONE process.

Checks first that both libraries produce the same pyramid bit for bit (reference-layout levels,
so tile padding cells do not count) on a set of shapes, then times the build at DSEC B=16 (and
AB_SHAPES) in rotated order.  Prints one line per (shape, library) and a JSON summary line.
  AB_ALT_LIB=tools/r1_lab/libecorr_r1.so python tools/ab_build.py
"""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402
from eraft_amd.layout import formats, untile  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SYMBOLS.items():
        try:
            fn = getattr(L, name)
        except AttributeError:   # an older library without a later symbol the build does not use
            continue
        fn.restype = res
        fn.argtypes = args
    assert L.ecorr_abi_version() >= 10, path   # the two-stage split build
    return L


LIBS = {"tree": load(_lib.LIB_PATH)}
# AB_ALT_LIB: path, or name=path,name=path,...
for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
    name, _, path = item.rpartition("=")
    LIBS[name or ("alt" if k == 0 else f"alt{k}")] = load(os.path.join(ROOT, path))
MODE = os.environ.get("AB_MODE", "split")


def levels_of(lib, f1, f2, levels=4):
    _lib._lib = lib
    B, D, H, W = f1.shape
    h, w, off = _lib.layout(B * H * W, H, W, levels)
    pyr = _lib.build_pyramid(f1, f2, B, D, H, W, H * W, levels, off, "ab build", mode=MODE)
    ntx = formats(H, W, levels)
    return [untile(pyr[off[i]:off[i + 1]], B * H * W, h[i], w[i], ntx[i], i) for i in range(levels)]


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    check = [(2, 256, 16, 24), (1, 256, 60, 80), (3, 100, 17, 22), (2, 64, 5, 300), (1, 256, 23, 40),
             (2, 256, 32, 32), (1, 3, 9, 13), (1, 256, 92, 160)]
    with torch.no_grad():
        if len(LIBS) > 1 and not os.environ.get("AB_NOCHECK"):
            # (shape, per-pixel 2^k scales with k in [-70, 50]: exponents outside the epilogue's
            # fast-scale window)
            for (B, D, H, W), wide in [(c, False) for c in check] + [((2, 256, 16, 24), True), ((1, 256, 60, 80), True)]:
                f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
                f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
                if wide:
                    for f in (f1, f2):
                        k = torch.randint(-70, 51, (B, 1, H, W), generator=g, device="cuda").float()
                        f.mul_(torch.exp2(k))
                lv = min(4, 1 + min((H).bit_length(), (W).bit_length()) - 2)
                ref = levels_of(LIBS[list(LIBS)[1]], f1, f2, lv)
                got = levels_of(LIBS["tree"], f1, f2, lv)
                for i in range(lv):
                    same = bool(((ref[i] == got[i]) | (ref[i].isnan() & got[i].isnan())).all())
                    print(f"bitwise {B}x{D}x{H}x{W}{' wide' if wide else ''} level {i}: {'same' if same else 'DIFFERENT'}", flush=True)
                    if not same:
                        d = (ref[i] - got[i]).abs().max().item()
                        raise SystemExit(f"pyramid differs at {B}x{D}x{H}x{W} level {i}: max |d| {d}")
        shapes = json.loads(os.environ.get("AB_SHAPES", "[[16, 256, 60, 80]]"))
        res = {}
        for (B, D, H, W) in shapes:
            f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
            f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
            times = {k: [] for k in LIBS}
            names = list(LIBS)
            for rnd in range(int(os.environ.get("AB_ROUNDS", "10"))):
                for name in names[rnd % len(names):] + names[:rnd % len(names)]:
                    _lib._lib = LIBS[name]
                    for _ in range(2):
                        eraft_amd.CorrBlock(f1, f2)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        eraft_amd.CorrBlock(f1, f2)
                    e1.record()
                    torch.cuda.synchronize()
                    times[name].append(e0.elapsed_time(e1) / 5)
            for name, ts in times.items():
                med = statistics.median(ts)
                print(f"build {B}x{D}x{H}x{W} {name:5s} median {med * 1e3:.1f} us  min {min(ts) * 1e3:.1f}", flush=True)
                res[f"{B}x{D}x{H}x{W}/{name}"] = round(med * 1e3, 1)
        print(json.dumps({"ab_build_us": res, "mode": MODE}))


if __name__ == "__main__":
    main()
