"""numpy front-end of the C oracle (oracle/ecorr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, never by the product package (e-raft_amd/).  See ecorr_oracle.c for the op orders restated
and the reference lines (model/corr.py, model/utils.py) each function follows.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libecorr_oracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def build():
    """Compile the oracle with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_corr_level0.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 6 + [_f32p]
        L.oracle_avg_pool2.argtypes = [_f32p, ctypes.c_long, ctypes.c_int, ctypes.c_int, _f32p]
        L.oracle_lookup.argtypes = [_f32p, _i64p, _i32p, _i32p, ctypes.c_int, ctypes.c_int, _f32p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p]
        L.oracle_bilinear_sampler.argtypes = [_f32p] + [ctypes.c_int] * 4 + [
            _f32p, ctypes.c_int, ctypes.c_int, _f32p, ctypes.c_void_p]
        L.oracle_coords_grid.argtypes = [ctypes.c_int] * 3 + [_f32p]
        L.oracle_grid_sample_values.argtypes = [_f32p, _f32p, ctypes.c_void_p, ctypes.c_int, ctypes.c_long,
                                                 ctypes.c_int, ctypes.c_int, _f32p, ctypes.c_void_p]
        L.oracle_forward_interpolate.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p]
        L.oracle_upsample_flow.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 4 + [_f32p]
        _u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
        _u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
        L.oracle_png16_encode.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u16p]
        L.oracle_png16_decode.argtypes = [_u16p, ctypes.c_long, _f32p, _u8p]
        L.oracle_png16_decode.restype = ctypes.c_int
        _f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
        L.oracle_voxel_dsec.argtypes = [_f32p] * 4 + [ctypes.c_long] + [ctypes.c_int] * 4 + [_f32p]
        L.oracle_voxel_dsec.restype = None
        L.oracle_voxel_mvsec.argtypes = [_f64p, ctypes.c_long] + [ctypes.c_int] * 4 + [_f32p]
        L.oracle_voxel_mvsec.restype = ctypes.c_int
        for fn in ("oracle_grid_sample_values", "oracle_forward_interpolate", "oracle_upsample_flow",
                   "oracle_png16_encode"):
            getattr(L, fn).restype = None
        for fn in ("oracle_corr_level0", "oracle_avg_pool2", "oracle_lookup",
                   "oracle_bilinear_sampler", "oracle_coords_grid"):
            getattr(L, fn).restype = None
        _lib = L
    return _lib


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def corr_level0(fmap1, fmap2, q_begin=0, q_count=None):
    """corr.py:52-60 as [B*q_count, H, W] (fp64-accumulated, then / sqrtf(D))."""
    f1, f2 = _c(fmap1), _c(fmap2)
    B, D, H, W = f1.shape
    Q = H * W
    q_count = Q - q_begin if q_count is None else q_count
    out = np.empty((B * q_count, H, W), dtype=np.float32)
    lib().oracle_corr_level0(f1, f2, B, D, H, W, q_begin, q_count, out)
    return out


def avg_pool2(x):
    """corr.py:26 F.avg_pool2d(x, 2, stride=2) on [N, h, w]."""
    x = _c(x)
    N, h, w = x.shape
    out = np.empty((N, h // 2, w // 2), dtype=np.float32)
    lib().oracle_avg_pool2(x, N, h, w, out)
    return out


def pyramid_from_level0(level0, num_levels=4):
    """corr.py:22-27: level 0 [N, h, w] followed by num_levels-1 pooled levels."""
    levels = [_c(level0)]
    for _ in range(num_levels - 1):
        h, w = levels[-1].shape[1:]
        if h // 2 < 1 or w // 2 < 1:
            raise RuntimeError("avg_pool2d: output size is too small")
        levels.append(avg_pool2(levels[-1]))
    return levels


def lookup(levels, coords, radius=4):
    """corr.py:29-50: levels = list of [B*H*W, h_i, w_i]; coords [B, 2, H, W] -> [B, C, H, W]."""
    coords = _c(coords)
    B, two, H, W = coords.shape
    assert two == 2
    L = len(levels)
    hs = np.array([lv.shape[1] for lv in levels], dtype=np.int32)
    ws = np.array([lv.shape[2] for lv in levels], dtype=np.int32)
    flat = np.concatenate([_c(lv).reshape(-1) for lv in levels])
    offs = np.zeros(L, dtype=np.int64)
    offs[1:] = np.cumsum([lv.size for lv in levels])[:-1]
    K = 2 * radius + 1
    out = np.empty((B, L * K * K, H, W), dtype=np.float32)
    lib().oracle_lookup(flat, offs, hs, ws, L, radius, coords, B, H, W, out)
    return out


def bilinear_sampler(img, coords, mask=False):
    """utils.py:7-21 with pixel coordinates; img [N,C,h,w], coords [N,Hg,Wg,2]."""
    img, coords = _c(img), _c(coords)
    N, C, h, w = img.shape
    _, Hg, Wg, _ = coords.shape
    out = np.empty((N, C, Hg, Wg), dtype=np.float32)
    m = np.empty((N, Hg, Wg, 1), dtype=np.float32) if mask else None
    lib().oracle_bilinear_sampler(img, N, C, h, w, coords, Hg, Wg, out,
                                  m.ctypes.data if mask else None)
    return (out, m) if mask else out


def coords_grid(batch, ht, wd):
    out = np.empty((batch, 2, ht, wd), dtype=np.float32)
    lib().oracle_coords_grid(batch, ht, wd, out)
    return out


def normwise_err(got, ref):
    """max|got - ref| / rms(ref): the GEMM parity statistic (tolerance 1e-5)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    rms = np.sqrt(np.mean(ref * ref))
    return float(np.max(np.abs(got - ref)) / rms)


def same_bits(a, b):
    """Bit-exact comparison modulo NaN payloads (x86 and gfx950 default NaNs differ)."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return bool(np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb]))


# ---- SURVEY §8f rows (next_oracle.c) ----

def forward_interpolate(flow):
    """image_utils.py:50-83: flow [B,2,h,w] (or [2,h,w]) -> [B,2,h,w]."""
    flow = _c(flow)
    if flow.ndim == 3:
        flow = flow[None]
    B, _, h, w = flow.shape
    out = np.empty_like(flow)
    lib().oracle_forward_interpolate(flow, B, h, w, out)
    return out


def grid_sample_values(inp, h, w):
    """image_utils.py:10-47: inp [3, n] -> (values [1,h,w] f32, valid [1,h,w] bool)."""
    inp = _c(inp).reshape(3, -1)
    n = inp.shape[1]
    values = np.empty((1, h, w), dtype=np.float32)
    valid = np.empty((1, h, w), dtype=np.uint8)
    z = inp[2].copy()
    lib().oracle_grid_sample_values(inp[0].copy(), inp[1].copy(), z.ctypes.data, 1, n, h, w, values,
                                    valid.ctypes.data)
    return values, valid.astype(bool)


def upsample_flow(flow, mask):
    """eraft.py:74-85: flow [N,2,H,W], mask [N,576,H,W] -> [N,2,8H,8W] (libm expf)."""
    flow, mask = _c(flow), _c(mask)
    N, _, H, W = flow.shape
    out = np.empty((N, 2, 8 * H, 8 * W), dtype=np.float32)
    lib().oracle_upsample_flow(flow, mask, N, H, W, 0, out)
    return out


def flow_to_png16(flow):
    """visualization.py:81-84: flow [2,h,w] or [B,2,h,w] -> uint16 [(B,) h, w, 3]."""
    f = _c(flow)
    single = f.ndim == 3
    if single:
        f = f[None]
    B, _, h, w = f.shape
    out = np.empty((B, h, w, 3), dtype=np.uint16)
    lib().oracle_png16_encode(f, B, h, w, out)
    return out[0] if single else out


def flow_16bit_to_float(png):
    """dsec_utils.py:66-83: uint16 [h,w,3] -> (flow [h,w,2] float32, valid [h,w] bool, n_bad)."""
    png = np.ascontiguousarray(png, dtype=np.uint16)
    h, w, _ = png.shape
    flow = np.empty((h, w, 2), dtype=np.float32)
    valid = np.empty((h, w), dtype=np.uint8)
    bad = lib().oracle_png16_decode(png, h * w, flow, valid)
    return flow, valid.astype(bool), bad


def voxel_dsec(p, t, x, y, C, H, W, normalize):
    """dsec_utils.py:26-64 -> [C, H, W] float32 (serial fold; normalization in double)."""
    p, t, x, y = (_c(v).reshape(-1) for v in (p, t, x, y))
    out = np.empty((C, H, W), dtype=np.float32)
    lib().oracle_voxel_dsec(p, t, x, y, p.size, C, H, W, int(bool(normalize)), out)
    return out


def voxel_mvsec(events, C, H, W, normalize):
    """transformers.py:36-126: events [n, 4] float64 -> ([C, H, W] float32, bad_index)."""
    ev = np.ascontiguousarray(events, dtype=np.float64)
    out = np.empty((C, H, W), dtype=np.float32)
    bad = lib().oracle_voxel_mvsec(ev, ev.shape[0], C, H, W, int(bool(normalize)), out)
    return out, bad
