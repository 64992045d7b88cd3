"""torch-CPU restatement of the reference CorrBlock -- the CPU baseline ("port") that bench.py times.

TEST/BASELINE INFRASTRUCTURE ONLY (see oracle/ecorr_oracle.c header): the reference Python cannot
travel to the GPU box, so bench.py's cpu_baseline leg times this restatement instead.  It issues
the same ATen ops as /root/reference/model/corr.py and model/utils.py, in the same order:
  build:  bmm(f1^T, f2) -> div by sqrt(D) (corr.py:52-60) -> 3 x avg_pool2d(2, 2) (corr.py:25-27)
  lookup: per level, CPU-built offset grid, coords / 2**i + offsets, pixel -> [-1, 1] mapping,
          grid_sample(align_corners=True) (utils.py:7-21), then cat + permute + contiguous
          (corr.py:35-50).
tests/test_torch_ref.py checks it bit-for-bit against the golden fixtures.
"""
import torch
import torch.nn.functional as F


class TorchCpuCorrBlock:
    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels, self.radius = num_levels, radius
        B, D, H, W = fmap1.shape
        a = fmap1.reshape(B, D, H * W).transpose(1, 2)
        vol = torch.bmm(a, fmap2.reshape(B, D, H * W))
        vol = vol / torch.sqrt(torch.tensor(D, dtype=torch.float32))
        lvl = vol.reshape(B * H * W, 1, H, W)
        self.corr_pyramid = [lvl]
        for _ in range(num_levels - 1):
            lvl = F.avg_pool2d(lvl, 2, stride=2)
            self.corr_pyramid.append(lvl)

    def __call__(self, coords):
        r = self.radius
        B, _, H, W = coords.shape
        c = coords.permute(0, 2, 3, 1).reshape(B * H * W, 1, 1, 2)
        k = 2 * r + 1
        steps = torch.linspace(-r, r, k).to(coords.device)   # corr.py:37-39 builds it on CPU, then .to()
        oy, ox = torch.meshgrid(steps, steps, indexing="ij")
        # last axis = (first meshgrid output, second) as in corr.py:39
        offs = torch.stack([oy, ox], dim=-1).view(1, k, k, 2)
        outs = []
        for i, img in enumerate(self.corr_pyramid):
            pts = c / 2 ** i + offs
            h, w = img.shape[-2:]
            px, py = pts[..., :1], pts[..., 1:]
            grid = torch.cat([2 * px / (w - 1) - 1, 2 * py / (h - 1) - 1], dim=-1)
            s = F.grid_sample(img, grid, align_corners=True)
            outs.append(s.view(B, H, W, -1))
        return torch.cat(outs, dim=-1).permute(0, 3, 1, 2).contiguous().float()


def grid_sample_values(input, height, width):
    """utils/image_utils.py:10-47, same ATen ops in the same order (ceil/floor, put_ accumulate)."""
    device = input.device
    ceil = torch.stack([torch.ceil(input[0, :]), torch.ceil(input[1, :]), input[2, :]])
    floor = torch.stack([torch.floor(input[0, :]), torch.floor(input[1, :]), input[2, :]])
    z = input[2, :].clone()
    values_ipl = torch.zeros(height * width, device=device)
    weights_acc = torch.zeros(height * width, device=device)
    for x_vals in [floor[0], ceil[0]]:
        for y_vals in [floor[1], ceil[1]]:
            m = (x_vals < width) & (x_vals >= 0) & (y_vals < height) & (y_vals >= 0)
            weights = (1 - (input[0] - x_vals).abs()) * (1 - (input[1] - y_vals).abs())
            idx = (x_vals + width * y_vals).long()
            values_ipl.put_(idx[m], (z * weights)[m], accumulate=True)
            weights_acc.put_(idx[m], weights[m], accumulate=True)
    valid = weights_acc.clone()
    valid[valid > 0] = 1
    valid = valid.bool().reshape([height, width])
    values = (values_ipl / (weights_acc + 1e-15)).reshape([height, width])
    return values.unsqueeze(0).clone(), valid.unsqueeze(0).clone()


def forward_interpolate_pytorch(flow_in):
    """utils/image_utils.py:50-83 (per-sample loop over the batch, as in the reference)."""
    flow = flow_in.clone()
    if len(flow.shape) < 4:
        flow = flow.unsqueeze(0)
    b, _, h, w = flow.shape
    device = flow.device
    dx, dy = flow[:, 0], flow[:, 1]
    y0, x0 = torch.meshgrid(torch.arange(0, h, 1), torch.arange(0, w, 1), indexing="ij")
    x0 = torch.stack([x0] * b).to(device)
    y0 = torch.stack([y0] * b).to(device)
    x1 = (x0 + dx).flatten(start_dim=1)
    y1 = (y0 + dy).flatten(start_dim=1)
    dx = dx.flatten(start_dim=1)
    dy = dy.flatten(start_dim=1)
    flow_new = torch.zeros(flow.shape, device=device)
    for i in range(b):
        flow_new[i, 0] = grid_sample_values(torch.stack([x1[i], y1[i], dx[i]]), h, w)[0]
        flow_new[i, 1] = grid_sample_values(torch.stack([x1[i], y1[i], dy[i]]), h, w)[0]
    return flow_new


def voxel_grid_dsec(events, C, H, W, normalize=True):
    """utils/dsec_utils.py:26-64 (VoxelGrid.convert), same ATen ops in the same order."""
    grid = torch.zeros((C, H, W), dtype=torch.float, device=events["p"].device)
    t = events["t"]
    t = (C - 1) * (t - t[0]) / (t[-1] - t[0])
    x0, y0, t0 = events["x"].int(), events["y"].int(), t.int()
    value = 2 * events["p"] - 1
    for xl in (x0, x0 + 1):
        for yl in (y0, y0 + 1):
            for tl in (t0, t0 + 1):
                m = (xl < W) & (xl >= 0) & (yl < H) & (yl >= 0) & (tl >= 0) & (tl < C)
                w = value * (1 - (xl - events["x"]).abs()) * (1 - (yl - events["y"]).abs()) * (1 - (tl - t).abs())
                idx = H * W * tl.long() + W * yl.long() + xl.long()
                grid.put_(idx[m], w[m], accumulate=True)
    if normalize:
        nz = torch.nonzero(grid, as_tuple=True)
        if nz[0].size()[0] > 0:
            mean, std = grid[nz].mean(), grid[nz].std()
            grid[nz] = (grid[nz] - mean) / std if std > 0 else grid[nz] - mean
    return grid


def voxel_grid_mvsec(events, C, H, W, normalize=True):
    """utils/transformers.py:36-126 (EventSequenceToVoxelGrid_Pytorch.__call__) on an [N, 4] float64
    (t, x, y, p) tensor already on its device, same ATen ops in the same order (the reference moves
    a numpy array to the device first; timed callers pass the device tensor)."""
    ev = events.clone()
    grid = torch.zeros(C, H, W, dtype=torch.float32, device=ev.device).flatten()
    last, first = ev[-1, 0], ev[0, 0]
    dt = last - first
    if dt == 0:
        dt = 1.0
    ev[:, 0] = (C - 1) * (ev[:, 0] - first) / dt
    ts, xs, ys = ev[:, 0], ev[:, 1].long(), ev[:, 2].long()
    pols = ev[:, 3].float()
    pols[pols == 0] = -1
    tis = torch.floor(ts)
    tis_long = tis.long()
    dts = ts - tis
    vals_left = pols * (1.0 - dts.float())
    vals_right = pols * dts.float()
    valid = (tis < C) & (tis >= 0)
    grid.index_add_(0, xs[valid] + ys[valid] * W + tis_long[valid] * W * H, vals_left[valid])
    valid = ((tis + 1) < C) & (tis >= 0)
    grid.index_add_(0, xs[valid] + ys[valid] * W + (tis_long[valid] + 1) * W * H, vals_right[valid])
    grid = grid.view(C, H, W)
    if normalize:
        nz = torch.nonzero(grid, as_tuple=True)
        if nz[0].size()[0] > 0:
            mean, std = grid[nz].mean(), grid[nz].std()
            grid[nz] = (grid[nz] - mean) / std if std > 0 else grid[nz] - mean
    return grid

