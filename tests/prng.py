"""Portable, bit-reproducible synthetic inputs for parity tests (test infrastructure).

Every value is produced by integer arithmetic (splitmix64) plus exact float64 sums, so the
same seed gives the same float32 bits on any host (this container, the GPU box, any libm).
The golden capture script (tests/golden/make_golden.py) and the GPU parity tests both
draw their inputs from here, which is why large DSEC-size inputs never need committing.

normal(seed, shape): Irwin-Hall(4) of 24-bit uniforms, rescaled to unit variance.
"""
import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n consecutive outputs of splitmix64 started at state `seed`."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _u24(seed: int, n: int) -> np.ndarray:
    """2n... uniforms k * 2^-24, k in [0, 2^24): two per 64-bit draw."""
    z = splitmix64(seed, (n + 1) // 2)
    hi = (z >> np.uint64(40)).astype(np.float64)
    lo = ((z >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.float64)
    u = np.empty(2 * z.size, dtype=np.float64)
    u[0::2] = hi
    u[1::2] = lo
    return u[:n] * (1.0 / 16777216.0)


def normal(seed: int, shape, scale: float = 1.0) -> np.ndarray:
    """float32 array of approximately N(0, scale^2) values, bit-reproducible."""
    n = int(np.prod(shape)) if len(shape) else 1
    u = _u24(seed, 4 * n).reshape(n, 4)
    s = (u[:, 0] + u[:, 1]) + (u[:, 2] + u[:, 3])  # exact in float64
    v = (s - 2.0) * 1.7320508075688772  # var(U)=1/12 -> 4/12 -> * sqrt(3)
    if scale != 1.0:
        v = v * scale
    return v.astype(np.float32).reshape(shape)


def uniform(seed: int, shape, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = _u24(seed, n)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def coords_with_flow(seed: int, B: int, H: int, W: int, sigma: float) -> np.ndarray:
    """coords_grid(B,H,W) + N(0, sigma^2) flow, as the reference's coords1 (eraft.py:120-123)."""
    ys, xs = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32),
                         indexing="ij")
    grid = np.stack([xs, ys])[None].repeat(B, axis=0)
    if sigma == 0.0:
        return np.ascontiguousarray(grid)
    return np.ascontiguousarray(grid + normal(seed, (B, 2, H, W), sigma))


def coords_smooth(seed: int, B: int, H: int, W: int, sigma: float = 9.0, jitter: float = 0.5) -> np.ndarray:
    """coords_grid + a smooth warm-start flow (5 x 5 box mean of N(0, sigma^2), zero-padded, /25 as
    avg_pool2d's count_include_pad) + N(0, jitter^2): the field shape of bench.py's coordinates."""
    n = normal(seed, (B, 2, H + 4, W + 4), sigma).astype(np.float64)
    n[:, :, :2] = 0.0
    n[:, :, -2:] = 0.0
    n[:, :, :, :2] = 0.0
    n[:, :, :, -2:] = 0.0
    c = np.cumsum(np.cumsum(np.pad(n, ((0, 0), (0, 0), (1, 0), (1, 0))), axis=2), axis=3)
    box = (c[:, :, 5:, 5:] - c[:, :, :-5, 5:] - c[:, :, 5:, :-5] + c[:, :, :-5, :-5]) / 25.0
    flow = box.astype(np.float32) + normal(seed + 1, (B, 2, H, W), jitter)
    return np.ascontiguousarray(coords_with_flow(0, B, H, W, 0.0) + flow)


def dsec_events(seed: int, n: int, H: int, W: int):
    """Synthetic DSEC events as the loader hands them to VoxelGrid.convert (loader_dsec.py:245-257):
    fp32 p in {0, 1}, t ascending from 0 (us), rectified x / y reaching slightly outside the image."""
    t = np.sort(uniform(seed, (n,), 0.0, 1e5)).astype(np.float32)
    t -= t[0]
    x = uniform(seed + 1, (n,), -1.5, W + 0.5)
    y = uniform(seed + 2, (n,), -1.5, H + 0.5)
    p = (uniform(seed + 3, (n,)) < 0.5).astype(np.float32)
    return p, t, x, y


def mvsec_events(seed: int, n: int, H: int, W: int):
    """Synthetic MVSEC event sequence features [n, 4] float64 (t ascending in s, integer x / y,
    p in {0, 1}), the input of EventSequenceToVoxelGrid_Pytorch."""
    t = np.sort(uniform(seed, (n,), 0.0, 1.0)).astype(np.float64) * 0.05 + 1400000000.0
    x = np.floor(uniform(seed + 1, (n,), 0.0, W)).astype(np.float64)
    y = np.floor(uniform(seed + 2, (n,), 0.0, H)).astype(np.float64)
    p = (uniform(seed + 3, (n,)) < 0.5).astype(np.float64)
    return np.ascontiguousarray(np.stack([t, x, y, p], 1))
