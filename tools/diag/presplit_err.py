# diagnostic: split vs presplit normwise error on the presplit test's "scales" case, per item
import sys, os, numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import prng, eraft_amd
DEV = "cuda:0"
for case in ("scales", "plain"):
    B, D, H, W, L, O = 2, 64, 24, 32, 4, 256
    f1 = prng.normal(261, (B, D, H, W)); f2 = prng.normal(262, (B, D, H, W))
    if case == "scales":
        f1 = (f1 * np.exp2(np.linspace(-20, 20, H * W)).reshape(1, 1, H, W)).astype(np.float32)
        f2 = (f2 * np.exp2(np.array([-30.0, 30.0]))[:, None, None, None]).astype(np.float32)
    f1, f2 = torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV)
    coords = torch.from_numpy(prng.coords_with_flow(263, B, H, W, 3.0)).to(DEV)
    w = torch.from_numpy(prng.normal(264, (O, 324)) * np.float32(0.05)).to(DEV)
    bias = torch.from_numpy(prng.normal(265, (O,)) * np.float32(0.1)).to(DEV)
    with torch.no_grad():
        blk = eraft_amd.CorrBlock(f1, f2)
        corr = blk(coords).double().cpu()
        ref = torch.relu(torch.einsum("oc,bchw->bohw", w.double().cpu(), corr) + bias.double().cpu()[None, :, None, None])
        for m in ("split", "presplit", "fused"):
            got = blk.lookup_conv1x1_relu(coords, w, bias, mode=m).double().cpu()
            d = (got - ref).abs()
            # per query relative error: max over o of |d| / rms over o of ref
            rq = d.amax(dim=1) / ref.pow(2).mean(dim=1).sqrt().clamp_min(1e-300)
            print(case, m, "normwise", float(d.max() / ref.pow(2).mean().sqrt()), "per-query max rel", float(rq.max()),
                  "median", float(rq.median()))
        sc = blk._colscale[:B * H * W].view(B, 1, H, W).cpu().double()
        s = corr.abs().amax(dim=1, keepdim=True) * torch.exp2(sc)
        print(case, "scaled column max: min", float(s.min()), "median", float(s.median()), "max", float(s.max()))
