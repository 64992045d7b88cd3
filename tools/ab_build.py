#!/usr/bin/env python3
"""Interleaved A/B timing of build-kernel variants in ONE process (cdna_hip_programming.md §5.4
rule 24).  Variants are selected through the dev-only env knobs read by launch_build."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402

VARIANTS = {
    "default": {},
    "regstage": {"ECORR_BUILD_GLDS": "0"},
}
# AB_VARIANTS='{"name": {"KNOB": "v", ...}, ...}' overrides; the pseudo-knob MODE picks the build
# mode (_lib.set_build_mode), the rest are the launch_build env knobs below
if os.environ.get("AB_VARIANTS"):
    import json
    VARIANTS = json.loads(os.environ["AB_VARIANTS"])
KNOBS = ("ECORR_BUILD_SKIP_EPILOGUE", "ECORR_BUILD_KB32", "ECORR_BUILD_NOBAND", "ECORR_BUILD_GLDS",
         "ECORR_BUILD_PK", "ECORR_BUILD_PACK2", "ECORR_BUILD_PKPIPE", "ECORR_BUILD_GM", "ECORR_BUILD_ABL")
B = int(os.environ.get("AB_BATCH", "16"))
H, W, D = 60, 80, 256
g = torch.Generator(device="cuda").manual_seed(0)
f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
flops = 2.0 * B * (H * W) ** 2 * D
times = {k: [] for k in VARIANTS}
ref = None
with torch.no_grad():
    names = list(VARIANTS)
    for rnd in range(int(os.environ.get("AB_ROUNDS", "8"))):
        # rotate the order every round: the first variant of a round runs measurably slower
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:
            env = dict(VARIANTS[name])
            eraft_amd._lib.set_build_mode(env.pop("MODE", "split"))
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(env)
            blk = eraft_amd.CorrBlock(f1, f2)   # warm
            torch.cuda.synchronize()
            if rnd == 0 and not {"ECORR_BUILD_SKIP_EPILOGUE", "ECORR_BUILD_ABL"} & set(VARIANTS[name]):   # every variant must produce a valid pyramid (pooling exact vs level 0)
                blk._levels_cache = None
                lv0, lv1 = blk.corr_pyramid[0][:64, 0], blk.corr_pyramid[1][:64, 0]
                p = (((lv0[:, 0::2, 0::2] + lv0[:, 0::2, 1::2]) + lv0[:, 1::2, 0::2]) + lv0[:, 1::2, 1::2]) * 0.25
                assert torch.equal(p, lv1), name
                if ref is None:
                    ref = blk.corr_pyramid[0][:4096].clone()
                err = (blk.corr_pyramid[0][:4096] - ref).abs().max().item()
                print(f"{name}: level-0 max |diff| vs first variant {err:.3g}", flush=True)
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                blk = eraft_amd.CorrBlock(f1, f2)
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1))
            del blk
for name, ts in times.items():
    med = statistics.median(ts)
    print(f"{name:10s} median {med:.3f} ms  min {min(ts):.3f}  -> {flops / med / 1e9:.1f} TFLOP/s "
          f"({flops / med / 1e9 / 157.3 * 100:.1f}% of 157.3)")
