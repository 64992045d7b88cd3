#!/usr/bin/env python3
"""Benchmark of the E-RAFT CorrBlock hot path on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: CorrBlock build (split-f16 or fp32 MFMA GEMM
+ fused pyramid; ECORR_BUILD_MODE) followed by the 12 GRU-iteration lookups, exactly the call pattern of ERAFT.forward
(eraft.py:107, 126-128), with inputs already resident in HBM.

  default (--mode batch): BASELINE configs[1] at N=1 -- DSEC 480x640 (fmaps 256 x 60 x 80), batch
      16 per GPU, warm-start coordinates (12 distinct coordinate fields = coords_grid + smooth
      flow + per-iteration jitter).  N>1 = configs[3]: one process per GPU, each with its own
      batch of pairs, no data-path collective ("weak" scaling).
  --mode rowshard: BASELINE configs[4] -- 1280x720 (fmap 256 x 92 x 160, padded 736 rows), batch
      4, query rows sharded over the N ranks, fmap2 row slabs all-gathered once per pair and the
      lookup output slabs once per iteration (one fixed-chunk all-gather each, RCCL; "strong"
      scaling).

    python bench.py [--gpus N --steps K --warmup W --batch 16 --no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

`--gpus N` always means N ranks: without a launcher (no WORLD_SIZE in the environment) and N > 1,
bench.py starts torch.distributed.run with N processes as a child and forwards its JSON line and
exit code; under a launcher whose WORLD_SIZE differs from N it exits non-zero.

Prints ONE JSON line on rank 0 with `roofline` (the dominant kernel, the split GEMM alone --
build_split16_kernel at D = 256 --
HIP events on its launch stream inside the timed region; `window_frac` = the whole build with its
operand pass; `traffic` = PMC HBM bytes from profiles/latest_pmc.json when its source digest
matches this tree), `kernels` (build, pack, lookup, build_fp32) and `cpu_baseline` (SURVEY 8(d):
the C1 shape, B = 1, build + 12 lookups on the GPU leg's first pair; the torch restatement of the
reference's ATen ops, oracle/torch_ref.py, on all host cores and on one core, and the C oracle;
median of 3 after a warm-up; rank 0 at N=1 only).
BENCH_SINGLE_DEVICE=1 puts every rank on cuda:0 with gloo (multi-process rehearsal on one GPU).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "flow pairs/sec (DSEC 480×640, 12 iters) at 1/8 GPUs; CorrBlock % roofline"
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix, spec (dense)
PEAK_F16_MFMA_TFLOPS = 2516.6   # MI355X_MICROARCH.md: BF16/F16 matrix, dense (1024 flop/clk/SIMD)
SPLIT_MFMA_PER_PRODUCT = 3      # split build: lo*hi + hi*lo + hi*hi on the f16 matrix cores
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak, spec


class TimingEvent:
    """A HIP timing event without the system-scope fence (hipEventDisableSystemFence): recording
    it does not write back and invalidate the caches between two kernels, which a default event
    (torch.cuda.Event) does -- about 5 us of idle GPU per record inside the timed region (rocprof
    trace, profiles/r03_final3). Timing only; the timed region is still closed by a synchronize.
    Calls the HIP runtime torch has already loaded (its path read from /proc/self/maps, so no
    second runtime can come in); TimingEvent.available() is False when it cannot be found, and the
    bench then falls back to torch.cuda.Event."""
    _hip = None
    DISABLE_SYSTEM_FENCE = 0x20000000

    @staticmethod
    def _runtime_path():
        try:
            with open("/proc/self/maps") as f:
                for line in f:
                    path = line.split()[-1] if len(line.split()) >= 6 else ""
                    if os.path.basename(path).startswith("libamdhip64.so"):
                        return path
        except OSError:
            pass
        return None

    @classmethod
    def available(cls):
        if cls._hip is None:
            import ctypes
            path = cls._runtime_path()
            if path is None:
                return False
            cls._hip = ctypes.CDLL(path)
        return True

    def __init__(self):
        import ctypes
        if not TimingEvent.available():
            raise RuntimeError("the HIP runtime torch loaded is not mapped in this process")
        self._ct = ctypes
        self.h = ctypes.c_void_p()
        rc = TimingEvent._hip.hipEventCreateWithFlags(ctypes.byref(self.h), ctypes.c_uint(self.DISABLE_SYSTEM_FENCE))
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags failed: {rc}")

    def record(self, stream=None):
        stream = stream if stream is not None else torch.cuda.current_stream()
        rc = TimingEvent._hip.hipEventRecord(self.h, self._ct.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed: {rc}")

    def elapsed_time(self, end):
        ms = self._ct.c_float()
        rc = TimingEvent._hip.hipEventElapsedTime(self._ct.byref(ms), self.h, end.h)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed: {rc}")
        return ms.value

    def destroy(self):
        if TimingEvent._hip is not None and self.h:
            TimingEvent._hip.hipEventDestroy(self.h)
            self.h = self._ct.c_void_p()

    def __del__(self):   # main() destroys them while the runtime is up; this is the fallback
        try:
            self.destroy()
        except Exception:
            pass


class TorchTimingEvent(torch.cuda.Event):
    """torch.cuda.Event with TimingEvent's interface (the fallback when no HIP runtime is mapped)."""

    def __init__(self):
        super().__init__(enable_timing=True)

    def destroy(self):
        pass


def timing_event():
    """A fence-free HIP timing event, or torch's own where the runtime path cannot be resolved."""
    return TimingEvent() if TimingEvent.available() else TorchTimingEvent()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=("batch", "rowshard"), default="batch")
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU (batch) / per job (rowshard)")
    ap.add_argument("--height", type=int, default=None, help="fmap rows")
    ap.add_argument("--width", type=int, default=None, help="fmap cols")
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-next", action="store_true", help="skip the SURVEY §8f next-row measurements")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end ERAFT.forward leg")
    a = ap.parse_args()
    if a.mode == "batch":
        a.batch, a.height, a.width = a.batch or 16, a.height or 60, a.width or 80
    else:
        a.batch, a.height, a.width = a.batch or 4, a.height or 92, a.width or 160
    return a


def algorithmic(B, D, H, W, L=4, r=4, q=None):
    """build flops 2*B*q*Q*D; build bytes 4*B*D*(q + Q) (fmaps in) + 4*B*q*sum(h_i*w_i)
    (pyramid out); lookup bytes B*q*[L(2r+2)^2*4 + L(2r+1)^2*4 + 8] (q = query pixels served,
    Q = H*W targets)."""
    Q = H * W
    q = Q if q is None else q
    flops = 2.0 * B * q * Q * D
    hs, ws, pix = H, W, 0
    for i in range(L):
        if i:
            hs, ws = hs // 2, ws // 2
        pix += hs * ws
    build_bytes = 4.0 * B * D * (q + Q) + 4.0 * B * q * pix
    look_bytes = B * q * (L * (2 * r + 2) ** 2 * 4 + L * (2 * r + 1) ** 2 * 4 + 2 * 4)
    return flops, build_bytes, look_bytes


def build_floors(flops, build_bytes, mode):
    """Ideal build time (s) on each roof: the matrix cores at the mode's rate, HBM for the bytes."""
    mfma_peak = PEAK_F16_MFMA_TFLOPS / SPLIT_MFMA_PER_PRODUCT if mode == "split" else PEAK_FP32_MFMA_TFLOPS
    return flops / (mfma_peak * 1e12), build_bytes / (PEAK_HBM_GBS * 1e9), mfma_peak


def make_inputs(B, D, H, W, iters, device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    f1 = torch.randn((B, D, H, W), generator=g, device=device)
    f2 = torch.randn((B, D, H, W), generator=g, device=device)
    import eraft_amd
    base = eraft_amd.coords_grid(B, H, W, device=device)
    # warm start: smooth initial flow (sigma ~3 px at 1/8 res) plus per-iteration refinement
    init = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device=device) * 9.0,
                                          5, stride=1, padding=2)
    coords = [(base + init + 0.5 * torch.randn((B, 2, H, W), generator=g, device=device)).contiguous()
              for _ in range(iters)]
    return f1, f2, coords


def cpu_baseline(f1, f2, coords, iters):
    """the reference's CPU path on this host's cores, at the C1 shape (B = 1, DSEC
    256 x 60 x 80, build + 12 lookups) on the GPU leg's own first pair (same PRNG inputs, copied to
    the host).  Two restatements of the reference, both bit-checked against its goldens:
      torch: oracle/torch_ref.py -- the reference's own ATen op sequence (corr.py, utils.py), on
             all cores and on 1 core (main.py:2-5 pins the reference to one thread);
      c:     oracle/ecorr_oracle.c -- the C restatement (fp64-accumulated GEMM), OpenMP on all cores.
    Each leg: one warm-up, then the median of 3 timed runs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from torch_ref import TorchCpuCorrBlock
    import oracle
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    a, b = f1[:1].cpu(), f2[:1].cpu()
    cs = [c[:1].cpu() for c in coords]
    an, bn, csn = a.numpy(), b.numpy(), [c.numpy() for c in cs]

    def med3(fn):
        fn()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[1]

    def torch_step():
        blk = TorchCpuCorrBlock(a, b)
        for c in cs:
            blk(c)

    def c_step():
        levels = oracle.pyramid_from_level0(oracle.corr_level0(an, bn), 4)
        for c in csn:
            oracle.lookup(levels, c, 4)

    nt = torch.get_num_threads()
    torch.set_num_threads(cores)
    t_all = med3(torch_step)
    torch.set_num_threads(1)
    t_one = med3(torch_step)
    torch.set_num_threads(nt)
    t_c = med3(c_step)   # OpenMP threads = OMP_NUM_THREADS (the box: 16)
    shape = f"B=1, fmap {a.shape[1]}x{a.shape[2]}x{a.shape[3]}, build + {iters} lookups"
    return {"value": round(1.0 / t_all, 3), "unit": "pairs/s", "cores": cores, "kind": "port",
            "batch": 1, "median_of": 3,
            "sample": f"C1: {shape}, the GPU leg's first pair; torch {torch.__version__} CPU ATen ops = the "
                      f"reference's op sequence (oracle/torch_ref.py), {cores} threads; median of 3 after a warm-up",
            "legs": {
                "torch_all_cores": {"pairs_per_s": round(1.0 / t_all, 3), "s_per_pair": round(t_all, 4), "cores": cores},
                "torch_1_core": {"pairs_per_s": round(1.0 / t_one, 3), "s_per_pair": round(t_one, 4), "cores": 1,
                                 "note": "torch.set_num_threads(1) as main.py:2-5"},
                "c_oracle": {"pairs_per_s": round(1.0 / t_c, 3), "s_per_pair": round(t_c, 4),
                             "cores": int(os.environ.get("OMP_NUM_THREADS", cores)),
                             "note": "oracle/ecorr_oracle.c, fp64-accumulated GEMM, OpenMP"}}}


def measure_fused_convc1(blk, coords, B, H, W, device, reps=3):
    """lookup + convc1 + ReLU (CorrBlock.lookup_conv1x1_relu) in both modes --
    "split" (the default: ecorr_lookup_qmax, then the split-f16 ecorr_conv1x1_relu_split) and "fused"
    (ecorr_lookup_conv1x1_relu_packed, one fp32-MFMA kernel) -- against the unfused path they replace
    (our lookup, then torch's conv2d + relu on MIOpen), 12 iterations, HIP events on the launch
    stream; outside the headline timed region.  `conv_split` times the split conv kernel alone on
    one materialized lookup (HBM-bound: corr in + out)."""
    import torch.nn.functional as F
    from eraft_amd import _lib
    g = torch.Generator(device=device).manual_seed(99)
    wgt = torch.randn((256, 324, 1, 1), generator=g, device=device) * 0.05
    bias = torch.randn((256,), generator=g, device=device) * 0.1
    stream = torch.cuda.current_stream(device)

    def run(fn, n=len(coords)):
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(n):
                fn(coords[i % len(coords)])
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / n)
        return sorted(ts[1:])[len(ts[1:]) // 2]

    Q = H * W
    with torch.no_grad():
        fused = run(lambda c: blk.lookup_conv1x1_relu(c, wgt, bias, mode="fused"))
        split = run(lambda c: blk.lookup_conv1x1_relu(c, wgt, bias, mode="split"))
        presplit = run(lambda c: blk.lookup_conv1x1_relu(c, wgt, bias, mode="presplit"))   # column scales: once
        presplit_ran = blk._colscale is not None
        unfused = run(lambda c: torch.relu(F.conv2d(blk(c), wgt, bias)))
        lookup = run(lambda c: blk(c))
        corr = torch.empty((B, 324, H, W), device=device)
        qmax = torch.empty((B, 12, Q), device=device)
        _lib.check(_lib.lib().ecorr_lookup_qmax(blk._pyramid.data_ptr(), coords[0].contiguous().data_ptr(), B, H, W,
                                                Q, 4, 4, corr.data_ptr(), qmax.data_ptr(), _lib.stream_of(corr)),
                   "lookup qmax")
        out = torch.empty((B, 256, H, W), device=device)
        pk = _lib.packed_conv1x1_weight(wgt, 256, 324, "split", _lib.stream_of(wgt), {})

        def conv_fn(qm):
            return lambda c: _lib.check(_lib.lib().ecorr_conv1x1_relu_split(
                corr.data_ptr(), B, 324, Q, None if qm is None else qm.data_ptr(), 12, pk.data_ptr(), bias.data_ptr(),
                256, out.data_ptr(), _lib.stream_of(corr)), "split conv")
        conv = run(conv_fn(qmax))
        conv_pre = run(conv_fn(None))
        conv_presplit = None
        if presplit_ran:   # the presplit conv alone on one presplit lookup (ABI 16)
            import ctypes
            nb = ctypes.c_int64()
            _lib.check(_lib.lib().ecorr_presplit_size(B, 4, Q, ctypes.byref(nb)), "presplit size")
            pin = torch.empty(nb.value, dtype=torch.uint8, device=device)
            _lib.check(_lib.lib().ecorr_lookup_presplit(blk._pyramid.data_ptr(), coords[0].contiguous().data_ptr(), B,
                                                        H, W, Q, 4, 4, blk._colscale.data_ptr(), pin.data_ptr(),
                                                        _lib.stream_of(pin)), "presplit lookup")
            pkp = _lib.packed_conv1x1_weight(wgt, 256, 324, "presplit", _lib.stream_of(wgt), {})
            conv_presplit = run(lambda c: _lib.check(_lib.lib().ecorr_conv1x1_relu_presplit(
                pin.data_ptr(), B, 4, Q, blk._colscale.data_ptr(), pkp.data_ptr(), bias.data_ptr(), 256,
                out.data_ptr(), _lib.stream_of(pin)), "presplit conv"))
    flops = 2.0 * B * Q * 256 * 324
    conv_bytes = 4.0 * B * Q * (324 + 256)
    default = os.environ.get("ECORR_CONVC1", "split")
    best = split if default == "split" else fused
    return {"mode": default, "ms_per_iter": round(best, 4),
            "split_ms_per_iter": round(split, 4), "fused_ms_per_iter": round(fused, 4),
            "presplit_ms_per_iter": round(presplit, 4) if presplit_ran else None,
            "presplit_conv_ms": round(conv_presplit, 4) if conv_presplit is not None else None,
            "presplit_note": "mode='presplit' (ABI 16): the lookup writes corr as f16 hi + lo under a per-query "
                             "bound scale, the conv loads it whole (no split, no maxima); not the default: the "
                             "lookup's split costs what the conv saves (DESIGN.md §3.3)",
            "unfused_ms_per_iter": round(unfused, 4), "lookup_ms_per_iter": round(lookup, 4),
            "speedup_vs_unfused": round(unfused / best, 3),
            "fp32_equiv": {"achieved": round(flops / (best * 1e-3) / 1e12, 2), "peak": PEAK_FP32_MFMA_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(flops / (best * 1e-3) / 1e12 / PEAK_FP32_MFMA_TFLOPS, 4),
                           "note": "the conv's 2*O*C flop per query over the whole lookup + convc1 time, "
                                   "against the fp32 MFMA peak (the split mode runs them as 3 f16 MFMAs each)"},
            "conv_split": {"ms": round(conv, 4), "ms_own_prepass": round(conv_pre, 4), "bound": "hbm",
                           "achieved": round(conv_bytes / (conv * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                           "unit": "GB/s", "frac": round(conv_bytes / (conv * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                           "bytes": f"{conv_bytes:.4g} B: corr in (324 x 4 B) + out (256 x 4 B) per query "
                                    "(+ 12 x 4 B of per-query maxima from ecorr_lookup_qmax; ms_own_prepass: "
                                    "without them, the kernel's own max pass re-reads corr)"},
            "work_per_launch": f"{flops:.4g} flop (1x1 conv 324->256 over B*H*W queries)"}


def measure_forward_interpolate(B, H, W, device, reps=5):
    """the warm-start splat (utils/image_utils.py:50-83) over the batch's
    [B, 2, H, W] low-res flow -- our one launch (splat.hip) against the reference's op sequence
    (oracle/torch_ref.py: per-sample loop of ATen put_ scatters) on this GPU and on the host CPU.
    Latency-bound: 16 B of algorithmic traffic per pixel (flow in, flow out)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch_ref
    import eraft_amd
    g = torch.Generator(device=device).manual_seed(5)
    flow = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device=device) * 9.0,
                                          5, stride=1, padding=2).contiguous()
    stream = torch.cuda.current_stream(device)

    def gpu_ms(fn):
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts[1:])[len(ts[1:]) // 2]

    ours = gpu_ms(lambda: eraft_amd.forward_interpolate_pytorch(flow))
    # the device's time per call: 10 calls captured into one HIP graph, replayed between two events
    # (the eager number above also holds the Python wrapper's host time before the launch)
    gph, per = torch.cuda.CUDAGraph(), 10
    with torch.cuda.graph(gph):
        for _ in range(per):
            eraft_amd.forward_interpolate_pytorch(flow)
    dev_ms = gpu_ms(gph.replay) / per
    del gph
    ref_gpu = gpu_ms(lambda: torch_ref.forward_interpolate_pytorch(flow))
    fc = flow.cpu()
    t0 = time.perf_counter()
    torch_ref.forward_interpolate_pytorch(fc)
    ref_cpu = (time.perf_counter() - t0) * 1e3
    return {"ms_per_call": round(ours, 4), "device_ms_per_call": round(dev_ms, 4), "batch": B, "flow": [2, H, W],
            "reference_ops_on_gpu_ms": round(ref_gpu, 3), "reference_ops_on_cpu_ms": round(ref_cpu, 3),
            "speedup_vs_reference_gpu": round(ref_gpu / ours, 1), "bound": "latency",
            "achieved_GBs": round(16.0 * B * H * W / (ours * 1e-3) / 1e9, 2),
            "note": "bit-exact with the reference's serial CPU put_; one launch for the whole batch"}


def measure_upsample(B, H, W, device, reps=5):
    """convex 8x upsampling (eraft.py:74-85) of a [B, 2, H, W] flow with its
    [B, 576, H, W] mask -- one HIP pass (upsample.hip) vs the reference's ATen expression on this
    GPU; HBM-bound: 2304 B of mask + 8 B of flow in, 512 B out per low-res pixel."""
    import eraft_amd
    import torch.nn.functional as F
    g = torch.Generator(device=device).manual_seed(6)
    flow = torch.randn((B, 2, H, W), generator=g, device=device) * 3.0
    mask = torch.randn((B, 576, H, W), generator=g, device=device) * 0.25
    stream = torch.cuda.current_stream(device)

    def ref():
        m = torch.softmax(mask.view(B, 1, 9, 8, 8, H, W), dim=2)
        up = F.unfold(8 * flow, [3, 3], padding=1).view(B, 2, 9, 1, 1, H, W)
        return torch.sum(m * up, dim=2).permute(0, 1, 4, 2, 5, 3).reshape(B, 2, 8 * H, 8 * W)

    def gpu_ms(fn, n=10):
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(n):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / n)
        return sorted(ts[1:])[len(ts[1:]) // 2]

    ours = gpu_ms(lambda: eraft_amd.upsample_flow(flow, mask))
    theirs = gpu_ms(ref)
    nbytes = B * H * W * (576 * 4 + 2 * 4 + 2 * 64 * 4)
    gbs = nbytes / (ours * 1e-3) / 1e9
    return {"ms_per_call": round(ours, 4), "reference_expr_on_gpu_ms": round(theirs, 4),
            "speedup": round(theirs / ours, 2), "bound": "hbm", "achieved": round(gbs, 1),
            "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
            "work_per_launch": f"{nbytes:.4g} B (mask + flow in, 8x flow out)"}


def measure_voxel(device, n=1_000_000, C=15, H=480, W=640, reps=5):
    """DSEC event -> voxel grid (dsec_utils.py:26-64) for one 100 ms window of
    n synthetic events at full resolution, normalized -- ours (voxel.hip: tile windows, a counting
    sort in LDS, ordered gather, normalization) vs the reference's ATen op sequence (oracle/torch_ref.py) on this
    GPU and on one host core (main.py pins torch to one thread)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch_ref
    import eraft_amd
    g = torch.Generator(device=device).manual_seed(8)
    t = torch.sort(torch.rand((n,), generator=g, device=device) * 1e5).values
    ev = {"p": (torch.rand((n,), generator=g, device=device) < 0.5).float(), "t": t - t[0],
          "x": torch.rand((n,), generator=g, device=device) * (W + 2) - 1.5,
          "y": torch.rand((n,), generator=g, device=device) * (H + 2) - 1.5}
    vg = eraft_amd.VoxelGrid((C, H, W), normalize=True)
    stream = torch.cuda.current_stream(device)

    def gpu_ms(fn):
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts[1:])[len(ts[1:]) // 2]

    ours = gpu_ms(lambda: vg.convert(ev))
    ref_gpu = gpu_ms(lambda: torch_ref.voxel_grid_dsec(ev, C, H, W))
    evc = {k: v.cpu() for k, v in ev.items()}
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    t0 = time.perf_counter()
    torch_ref.voxel_grid_dsec(evc, C, H, W)
    ref_cpu = (time.perf_counter() - t0) * 1e3
    torch.set_num_threads(nt)
    # algorithmic bytes: the four event fields in (fp32) + the grid out, once each
    nbytes = 16.0 * n + 4.0 * C * H * W
    gbs = nbytes / (ours * 1e-3) / 1e9
    return {"ms_per_call": round(ours, 4), "events": n, "grid": [C, H, W],
            "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4),
            "work_per_launch": f"{nbytes:.4g} B (events in + grid out; the bucketing of the events into "
                               "tile windows, 1.33 copies each, and the windows' reads are not algorithmic bytes)",
            "events_per_s": round(n / (ours * 1e-3), 1),
            "reference_ops_on_gpu_ms": round(ref_gpu, 3), "reference_ops_on_1_cpu_core_ms": round(ref_cpu, 1),
            "speedup_vs_reference_gpu": round(ref_gpu / ours, 2),
            "note": "accumulated grid bit-exact with the reference's serial fold (the reference on a "
                    "GPU uses float atomics: not reproducible); normalization within 1e-6"}


def measure_voxel_mvsec(device, n=300_000, C=15, H=260, W=346, reps=5):
    """SURVEY §8f row 3, MVSEC form: EventSequenceToVoxelGrid_Pytorch (transformers.py:36-126) on
    n synthetic events [n, 4] float64 already on the device (the reference moves a numpy array
    there first; both legs here start from the device tensor), normalized -- ours (voxel.hip's
    key-range counting sort and ordered gather, bit-exact) vs the reference's ATen ops
    (oracle/torch_ref.py: index_add_ with float atomics) on this GPU and on one host core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch_ref
    import eraft_amd
    g = torch.Generator(device=device).manual_seed(9)
    t = torch.sort(torch.rand((n,), generator=g, device=device, dtype=torch.float64)).values * 0.05 + 1.4e9
    ev = torch.stack([t, torch.floor(torch.rand((n,), generator=g, device=device, dtype=torch.float64) * W),
                      torch.floor(torch.rand((n,), generator=g, device=device, dtype=torch.float64) * H),
                      (torch.rand((n,), generator=g, device=device) < 0.5).double()], 1).contiguous()

    class _Seq:
        features, image_width, image_height = ev, W, H
    conv = eraft_amd.EventSequenceToVoxelGrid_Pytorch(C, gpu=True, normalize=True)
    stream = torch.cuda.current_stream(device)

    def gpu_ms(fn):
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts[1:])[len(ts[1:]) // 2]

    ours = gpu_ms(lambda: conv(_Seq))
    ref_gpu = gpu_ms(lambda: torch_ref.voxel_grid_mvsec(ev, C, H, W))
    evc = ev.cpu()
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    t0 = time.perf_counter()
    torch_ref.voxel_grid_mvsec(evc, C, H, W)
    ref_cpu = (time.perf_counter() - t0) * 1e3
    torch.set_num_threads(nt)
    nbytes = 32.0 * n + 4.0 * C * H * W   # the events in (4 x fp64) + the grid out
    gbs = nbytes / (ours * 1e-3) / 1e9
    return {"ms_per_call": round(ours, 4), "events": n, "grid": [C, H, W],
            "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4),
            "work_per_launch": f"{nbytes:.4g} B (events in + grid out)",
            "reference_ops_on_gpu_ms": round(ref_gpu, 3), "reference_ops_on_1_cpu_core_ms": round(ref_cpu, 1),
            "speedup_vs_reference_gpu": round(ref_gpu / ours, 2),
            "note": "includes the wrapper's out-of-range check (one host sync, as the reference's index_add_ "
                    "raises); accumulated grid bit-exact with the reference's serial index_add_"}


def shape_key(B, D, H, W, q):
    """The launch shape a PMC record belongs to: batch, feature width, query pixels per pair (the
    slab, row-shard mode), target map."""
    return f"B{B}_D{D}_q{q}_{H}x{W}"


def pmc_traffic(kernel_prefix, key, path=None):
    """HBM bytes per dispatch of the dominant kernel from the committed PMC summary
    (profiles/latest_pmc.json, tools/pmc_summary.py), keyed by launch shape: used only when the
    summary's kernel-source digest is this tree's AND it holds a record of this very shape (a
    summary of other kernels or of another config is refused, not reported)."""
    import eraft_amd
    path = path or os.path.join(ROOT, "profiles", "latest_pmc.json")
    try:
        js = json.load(open(path))
    except (OSError, ValueError):
        return None, "no profiles/latest_pmc.json"
    here = eraft_amd._lib.source_digest()
    if js.get("source_digest") != here:
        return None, f"refused: profiles/latest_pmc.json measured sources {js.get('source_digest')}, tree is {here}"
    shapes = js.get("shapes", {})
    if key not in shapes:
        return None, f"refused: shape {key} not profiled (profiled: {sorted(shapes)})"
    for name, rec in shapes[key].get("kernels", {}).items():
        if name.startswith(kernel_prefix) and "hbm_bytes" in rec:
            return rec["hbm_bytes"], (f"{js.get('source', path)}: {name} at {key} ({rec.get('read_correction')}), "
                                      f"sources {here}")
    return None, f"no {kernel_prefix} record at {key} in profiles/latest_pmc.json"


def measure_lookup_fields(blk, B, H, W, iters, look_bytes, device, reps=3):
    """SURVEY 8(d)'s coordinate fields beside the bench's smooth warm-start one: coords_grid + i.i.d.
    N(0, 3 px) flow (the primary synthetic input) and the sigma = 40 px stress field (mostly out of
    bounds); `iters` distinct fields each, 12 lookups between two HIP events on the launch stream,
    median of reps after a warm-up, outside the headline timed region."""
    import eraft_amd
    g = torch.Generator(device=device).manual_seed(77)
    base = eraft_amd.coords_grid(B, H, W, device=device)
    stream = torch.cuda.current_stream(device)
    res = {}
    for name, sigma in (("lookup_iid", 3.0), ("lookup_stress", 40.0)):
        cs = [(base + sigma * torch.randn((B, 2, H, W), generator=g, device=device)).contiguous()
              for _ in range(iters)]
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for c in cs:
                blk(c)
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / iters)
        ms = sorted(ts[1:])[len(ts[1:]) // 2]
        gbs = look_bytes / (ms * 1e-3) / 1e9
        res[name] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(gbs / PEAK_HBM_GBS, 4), "ms_per_launch": round(ms, 4),
                     "coords": f"coords_grid + i.i.d. N(0, {sigma:g} px) flow, {iters} fields"}
    return res


def measure_e2e(B, iters, device, reps=5):
    """BASELINE's literal metric, end to end: ERAFT.forward (eraft_amd.network, the reference's
    module tree and call pattern, eraft.py:88-145) at DSEC 480x640 (15-bin voxel pairs, fmaps
    D x 60 x 80), batch B, `iters` GRU iterations, warm start (flow_init = a smooth low-res flow),
    PRNG weights at the reference's init scales (tests/e2e_weights.py; the checkpoints are
    download-only).  Median of `reps` forwards after a warm-up, outside the headline timed region,
    for (a) the reference's CorrBlock op sequence on the GPU (bmm, avg_pool2d, grid_sample:
    oracle/torch_ref.py, a reference leg), (b) eraft_amd.CorrBlock in the reference's call pattern,
    (c) (b) + the HIP lookup + convc1 + ReLU (CorrBlock.lookup_conv1x1_relu in its default mode,
    `convc1_mode`; the key keeps its round-3 name) and the HIP convex upsampling; with the CorrBlock
    share of each forward (build + iters lookups of that CorrBlock -- for (c) the lookup + convc1 --
    timed alone on the same fmaps)."""
    import statistics
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import eraft_amd
    import eraft_amd.network as nw
    from e2e_weights import make_state_dict
    from torch_ref import TorchCpuCorrBlock
    torch.backends.cudnn.benchmark = True
    g = torch.Generator(device=device).manual_seed(4321)
    im1 = torch.randn((B, 15, 480, 640), generator=g, device=device)
    im2 = torch.randn((B, 15, 480, 640), generator=g, device=device)
    yy, xx = torch.meshgrid(torch.arange(60, device=device, dtype=torch.float32),
                            torch.arange(80, device=device, dtype=torch.float32), indexing="ij")
    flow0 = torch.stack([2.0 * torch.sin(yy / 9.0), 1.5 * torch.cos(xx / 11.0)]).expand(B, 2, 60, 80).contiguous()
    stream = torch.cuda.current_stream(device)

    def net_of(fuse=False, hip_up=False):
        net = nw.ERAFT({"subtype": "warm_start"}, n_first_channels=15, fuse_motion_corr=fuse, hip_upsample=hip_up)
        net.load_state_dict(make_state_dict(net.state_dict()))
        return net.eval().to(device)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    res = {"config": f"DSEC 480x640, 15 bins, batch {B}, {iters} iterations, warm start, PRNG weights",
           "covers": "ERAFT.forward (encoders, CorrBlock, GRU update block, upsampling) between two HIP "
                     "events, median of %d after a warm-up" % reps}
    with torch.no_grad():
        base = net_of()
        fm1, fm2 = base.fnet([base.image_padder.pad(im1).contiguous(), base.image_padder.pad(im2).contiguous()])
        fm1, fm2 = fm1.float().contiguous(), fm2.float().contiguous()
        c1 = eraft_amd.coords_grid(B, 60, 80, device=device) + flow0

        def corr_only(cls, fused):
            conv = base.update_block.encoder.convc1

            def run():
                blk = cls(fm1, fm2, num_levels=4, radius=4)
                for _ in range(iters):
                    if fused:
                        blk.lookup_conv1x1_relu(c1, conv.weight, conv.bias)
                    else:
                        blk(c1)
            return run
        legs = (("reference_corrblock_ops_on_gpu", base, TorchCpuCorrBlock, False),
                ("eraft_amd_corrblock", base, None, False),
                ("eraft_amd_corrblock_fused_convc1_hip_upsample", net_of(True, True), None, True))
        saved = nw.CorrBlock
        for name, net, cls, fused in legs:
            try:
                if cls is not None:
                    nw.CorrBlock = cls
                ms = timed(lambda: net(im1, im2, iters=iters, flow_init=flow0))
            finally:
                nw.CorrBlock = saved
            corr_ms = timed(corr_only(cls or eraft_amd.CorrBlock, fused))
            res[name] = {"ms_per_forward": round(ms, 3), "pairs_per_s": round(B / (ms * 1e-3), 2),
                         "corrblock_ms": round(corr_ms, 3), "corrblock_share": round(corr_ms / ms, 4)}
            if fused:
                res[name]["convc1_mode"] = os.environ.get("ECORR_CONVC1", "split")
        del fm1, fm2
    res["speedup_vs_reference_corrblock"] = round(res["reference_corrblock_ops_on_gpu"]["ms_per_forward"] /
                                                  res["eraft_amd_corrblock"]["ms_per_forward"], 3)
    torch.cuda.empty_cache()
    return res


def measure_fp32_step(make_block, coords, B, iters, ideal_s, reps=5):
    """North star's literal fp32-MFMA configuration as a whole step (ecorr_build, build_f32_kernel,
    + the 12 lookups), outside the headline timed region: reps steps between two HIP events on the
    launch stream after a warm-up step, the build mode restored afterwards."""
    import eraft_amd
    prev = eraft_amd._lib.build_mode()
    eraft_amd._lib.set_build_mode("fp32")
    try:
        stream = torch.cuda.current_stream()

        def step():
            blk = make_block()
            for c in coords:
                blk(c)
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            step()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
    finally:
        eraft_amd._lib.set_build_mode(prev)
    return {"pairs_per_s": round(B / (ms * 1e-3), 2), "ms_per_step": round(ms, 4), "steps": reps,
            "corrblock_frac": round(ideal_s / (ms * 1e-3), 4), "mode": "fp32",
            "covers": f"ecorr_build (build_f32_kernel, v_mfma_f32_32x32x2_f32) + {iters} lookups per step",
            "ideal": "fp32-MFMA roof for the build + the lookups at 8 TB/s"}


def measure_pack(f1, f2, B, D, H, W, q, stream, reps=20):
    """The split build's operand pass (pack_both_kernel) alone, after the timed region (whose steps
    record events around the GEMM only): `reps` back-to-back launches between two HIP events on the
    launch stream -- kernel boundaries as inside a step, no event between the launches -- per
    launch, the median of 3 such bursts."""
    import ctypes
    import eraft_amd
    L = eraft_amd._lib.lib()
    n = ctypes.c_int64()
    eraft_amd._lib.check(L.ecorr_build_split_workspace_size(B, D, H, W, q, ctypes.byref(n)), "pack ws")
    ws = torch.empty(n.value, dtype=torch.uint8, device=f1.device)
    st = eraft_amd._lib.stream_of(f1)

    def launch():
        eraft_amd._lib.check(L.ecorr_build_split_pack(f1.data_ptr(), f2.data_ptr(), B, D, H, W, q, ws.data_ptr(),
                                                      st), "pack")
    # the practical roof of a pass that reads the fmaps once and writes as many bytes: the runtime's
    # device copy of both fmaps into scratch (f16 hi + lo = the fp32 bytes), timed the same way
    s1 = f1.reshape(-1)[:B * D * q]   # the query side's bytes (a row slab holds q = rows x W queries)
    d1, d2 = torch.empty_like(s1), torch.empty_like(f2)

    def copy():
        d1.copy_(s1)
        d2.copy_(f2)

    def burst(fn, n):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(3):
            e0, e1 = timing_event(), timing_event()
            e0.record(stream)
            for _ in range(n):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / n)
            e0.destroy()
            e1.destroy()
        return sorted(ts)[1]
    pack_ms, copy_ms = burst(launch, reps), burst(copy, reps)
    del d1, d2, s1
    return pack_ms, copy_ms


def measure_fp32_build(f1, f2, reps=5, per=3):
    """The fp32-MFMA build (ecorr_build: v_mfma_f32_32x32x2_f32, an exact fmaf chain per element)
    on the same inputs, outside the headline timed region: `per` back-to-back launches into one
    preallocated pyramid between two HIP events on the launch stream (host gaps amortized), median
    of reps after a warm-up."""
    from eraft_amd import _lib
    B, D, H, W = f1.shape
    _, _, off = _lib.layout(B * H * W, H, W, 4)
    stream = torch.cuda.current_stream(f1.device)
    pyr = torch.empty(off[-1], dtype=torch.float32, device=f1.device)
    st = _lib.stream_of(f2)

    def launch():
        _lib.check(_lib.lib().ecorr_build(f1.data_ptr(), f2.data_ptr(), B, D, H, W, H * W, 4, pyr.data_ptr(), st),
                   "fp32 build")
    launch()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(per):
            launch()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / per)
    del pyr
    ms = sorted(ts)[len(ts) // 2]
    flops = 2.0 * B * (H * W) ** 2 * D
    tf = flops / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / PEAK_FP32_MFMA_TFLOPS, 4), "ms_per_launch": round(ms, 4),
            "mode": "fp32", "covers": "build_f32_kernel (D = 256: v_mfma_f32_32x32x2_f32, fp32 operands straight "
                                      "from the fmaps, one launch)",
            "note": "north_star's fp32-MFMA design; the headline uses the split build (more accurate vs fp64, "
                    "tests/test_build_modes_gpu.py)"}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` (N > 1) with no launcher around it: start N ranks under
    torch.distributed.run as a CHILD process (never exec -- this process has not touched the GPU,
    but the ranks will) and return its exit code; rank 0's single JSON line reaches our stdout
    through the inherited descriptor."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    sys.stdout.flush()
    return subprocess.run(cmd, cwd=ROOT).returncode


def main():
    a = parse()
    if a.gpus < 1:
        raise SystemExit(f"--gpus {a.gpus}: need at least one rank")
    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:   # before any GPU call in this process
            raise SystemExit(launch_ranks(a.gpus))
    elif int(os.environ["WORLD_SIZE"]) != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: launch N ranks "
                         f"for --gpus N (or run `python bench.py --gpus N` alone and it launches them)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    single = os.environ.get("BENCH_SINGLE_DEVICE") == "1"
    dev_index = 0 if single else local
    device = torch.device("cuda", dev_index)
    torch.cuda.set_device(device)
    distributed = world > 1 or a.mode == "rowshard"
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")   # plain `python bench.py --mode rowshard`
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        backend = "gloo" if single else "nccl"
        kw = {} if single else {"device_id": device}
        dist.init_process_group(backend, **kw)
    import eraft_amd

    B, D, H, W, iters = a.batch, a.dim, a.height, a.width, a.iters
    stream = torch.cuda.current_stream(device)
    if a.mode == "batch":
        f1, f2, coords = make_inputs(B, D, H, W, iters, device, seed=1234 + rank)

        def make_block():
            return eraft_amd.CorrBlock(f1, f2, num_levels=4, radius=4)
        q_local = H * W
    else:
        from eraft_amd.rowshard import RowShardedCorrBlock, row_partition
        f1, f2, coords = make_inputs(B, D, H, W, iters, device, seed=1234)   # same job on every rank
        starts, counts = row_partition(H, world)
        r0, rr = starts[rank], counts[rank]
        f1_rows = f1[:, :, r0:r0 + rr].contiguous()
        f2_rows = f2[:, :, r0:r0 + rr].contiguous()

        def make_block():
            return RowShardedCorrBlock.from_row_slabs(f1_rows, f2_rows, H)
        q_local = rr * W

    # every event record in the stream leaves a ~5 us gap between kernels (rocprof trace,
    # profiles/r02_final7): with the split build in batch mode its own stage events (before the
    # operand pass, between the two launches, after the GEMM) bracket the build, and a step's
    # lookups end where the next step's operand pass begins, so only the last step records an
    # event after its lookups
    lean = a.mode == "batch" and eraft_amd._lib.build_mode() == "split"

    def step(ev=None, last=True):
        if ev is not None and not lean:
            ev[0].record(stream)
        blk = make_block()
        if ev is not None and not lean:
            ev[1].record(stream)
        for c in coords:
            blk(c)
        if ev is not None and (last or not lean):
            ev[2].record(stream)
        return blk

    with torch.no_grad():
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        evs = [[timing_event() for _ in range(3)] for _ in range(a.steps)]
        eraft_amd._lib.stage_events = stages = []   # split build: events around its GEMM launch
        eraft_amd._lib.stage_event = timing_event
        eraft_amd._lib.stage_event_start = not lean   # lean: the operand pass is timed after the loop
        t0 = time.perf_counter()
        for k in range(a.steps):
            step(evs[k], last=k == a.steps - 1)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        eraft_amd._lib.stage_events = None
        eraft_amd._lib.stage_event = None
        eraft_amd._lib.stage_event_start = True

    if lean:
        if len(stages) != a.steps:
            raise RuntimeError(f"{len(stages)} split builds recorded for {a.steps} timed steps")
        # two events per timed step, around the GEMM; the operand pass is timed after the loop
        # (measure_pack) and taken out of the interval from a GEMM's end to the next step's GEMM
        # start (its 12 lookups + the next operand pass); the last step closes with its own event
        with torch.no_grad():
            pack_ms, copy_ms = measure_pack(f1, f2, B, D, H, W, q_local, stream)
        gemm_each = [e[1].elapsed_time(e[2]) for e in stages]
        build_ms = sum(gemm_each) / a.steps + pack_ms
        inter = [stages[k][2].elapsed_time(stages[k + 1][1]) - pack_ms for k in range(a.steps - 1)] + \
                [stages[-1][2].elapsed_time(evs[-1][2])]
        look_each = [x / iters for x in inter]
        look_ms = sum(inter) / a.steps / iters
        step_each = [g + x + pack_ms for g, x in zip(gemm_each, inter)]
    else:
        build_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / a.steps
        look_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / a.steps / iters
    if not lean:
        look_each = [e[1].elapsed_time(e[2]) / iters for e in evs]
        step_each = [e[0].elapsed_time(e[2]) for e in evs]
    if not lean:
        gemm_each = [e[1].elapsed_time(e[2]) for e in stages] if stages else []
        pack_ms = sum(e[0].elapsed_time(e[1]) for e in stages) / len(stages) if stages else 0.0
    gemm_ms = sum(e[1].elapsed_time(e[2]) for e in stages) / len(stages) if stages else build_ms
    for ev in evs + stages:
        for e in ev:
            if e is not None:
                e.destroy()
    if distributed:
        t = torch.tensor([elapsed, build_ms, look_ms, pack_ms, gemm_ms], dtype=torch.float64,
                         device="cpu" if single else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, build_ms, look_ms, pack_ms, gemm_ms = t.tolist()

    flops, build_bytes, look_bytes = algorithmic(B, D, H, W, q=q_local)
    mode = eraft_amd._lib.build_mode()
    t_mfma, t_hbm, mfma_peak = build_floors(flops, build_bytes, mode)
    note = "" if a.mode == "batch" else " (per rank; lookup time includes the output all-gather)"

    def roofs(ms):
        tf, gbs = flops / (ms * 1e-3) / 1e12, build_bytes / (ms * 1e-3) / 1e9
        m = {"bound": "mfma", "achieved": round(tf, 2), "peak": round(mfma_peak, 1), "unit": "TFLOP/s",
             "frac": round(tf / mfma_peak, 4), "work_per_launch": f"{flops:.4g} flop" + note}
        h = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
             "frac": round(gbs / PEAK_HBM_GBS, 4),
             "work_per_launch": f"{build_bytes:.4g} B (fmaps in + pyramid out)" + note}
        # binding roof = the longer ideal time (split: HBM, the 1.96 GB pyramid store outweighs 3 f16
        # MFMAs per product; fp32: the fp32 matrix cores)
        return (m, h) if t_mfma >= t_hbm else (h, m)

    look_gbs = look_bytes / (look_ms * 1e-3) / 1e9
    kernels = {}
    # the split GEMM kernel: v_mfma_f32_16x16x32_f16 at D = 256 (E-RAFT), the 32x32x16 kernel otherwise
    split_kernel = "build_split16_kernel" if D == 256 else "build_split_kernel"
    if mode == "split":
        bind, other = roofs(gemm_ms)
        wbind, _ = roofs(build_ms)
        kernels["build"] = dict(bind, ms_per_launch=round(gemm_ms, 4), mode=mode,
                                covers=f"{split_kernel} alone (GEMM + fused pyramid; HIP events on the launch stream "
                                       "around its launch inside the timed region)",
                                other_roof={k: other[k] for k in ("bound", "achieved", "peak", "unit", "frac")},
                                window={"ms": round(build_ms, 4), "frac": wbind["frac"], "achieved": wbind["achieved"],
                                        "covers": f"pack_both_kernel + {split_kernel} (the whole CorrBlock build)"})
        kernels["pack"] = {"ms_per_launch": round(pack_ms, 4),
                           "covers": "pack_both_kernel (operand pass)" + (": 20 back-to-back launches between two "
                                     "events after the timed region, median of 3" if lean else ""),
                           "bound": "hbm", "work_per_launch": f"{4.0 * B * D * (q_local + H * W) * 2:.4g} B "
                                                             "(fmaps in, f16 hi/lo panels out)"}
        if lean:
            kernels["pack"]["copy_same_bytes_ms"] = round(copy_ms, 4)
            kernels["pack"]["copy_covers"] = ("torch copy_ of both fmaps into scratch (reads and writes the "
                                              "pass's bytes), timed as the pack")
    else:
        bind, other = roofs(build_ms)
        kernels["build"] = dict(bind, ms_per_launch=round(build_ms, 4), mode=mode, covers="build_kernel",
                                other_roof={k: other[k] for k in ("bound", "achieved", "peak", "unit", "frac")})
    kernels["lookup"] = {"bound": "hbm", "achieved": round(look_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(look_gbs / PEAK_HBM_GBS, 4), "ms_per_launch": round(look_ms, 4),
                         "launches_per_step": iters, "work_per_launch": f"{look_bytes:.4g} B" + note,
                         "covers": ("a step's 12 lookups / 12: from its GEMM's end event to the next step's "
                                    "GEMM-start event minus the operand pass (kernels.pack; the last step: to its "
                                    "closing event) -- kernel boundaries and host gaps included" if lean else
                                    "a step's 12 lookups / 12 between two HIP events")}
    if lean:   # the lookup share is an estimate (the pack burst-timed after the loop)
        kernels["lookup"]["estimate"] = ("pack-subtracted: kernels.pack is timed in warm back-to-back bursts "
                                         "after the timed region, not inside each step; tools/lk_percall.py "
                                         "times each call between its own events")

    def spread_seq(xs):   # min / median / max and the first and last of the sequence
        if not xs:
            return None
        ys = sorted(xs)
        return {"min": round(ys[0], 4), "median": round(ys[len(ys) // 2], 4), "max": round(ys[-1], 4),
                "first": round(xs[0], 4), "last": round(xs[-1], 4)}
    # per timed step (this rank): the clock settles over the first ~15 steps of sustained load
    # (DESIGN.md §5), so the spread shows where in that transient the driver's steps sit
    kernels["per_step"] = {"steps": a.steps, "step_ms": spread_seq(step_each),
                           "lookup_ms_per_call": spread_seq(look_each),
                           "covers": "HIP events of the timed region (lean: GEMM + its 12 lookups + "
                                     "kernels.pack, a pack-subtracted estimate); lookup = its 12 calls / 12"}
    if gemm_each:
        kernels["build"]["per_step_ms"] = spread_seq(gemm_each)
    if mode == "split" and a.mode == "batch" and world == 1 and not a.no_next:
        with torch.no_grad():
            kernels["build_fp32"] = measure_fp32_build(f1, f2)
    dom = "build" if gemm_ms >= look_ms * iters else "lookup"
    roof = {k: kernels[dom][k] for k in ("bound", "achieved", "peak", "unit", "frac")}
    roof["kernel"] = split_kernel if (dom == "build" and mode == "split") else \
        ("build_kernel" if dom == "build" else "lookup_cols_reg")
    if dom == "build" and mode == "split":
        roof["window_frac"] = kernels["build"]["window"]["frac"]
    key = shape_key(B, D, H, W, q_local)
    traffic, src = pmc_traffic(roof["kernel"], key)
    roof["shape_key"] = key
    roof["traffic"] = traffic
    roof["traffic_source"] = src
    ideal_s = max(t_mfma, t_hbm) + iters * look_bytes / (PEAK_HBM_GBS * 1e9)
    if a.mode == "batch" and not a.no_next:
        with torch.no_grad():
            kernels.update(measure_lookup_fields(make_block(), B, H, W, iters, look_bytes, device))
    if mode == "split" and a.mode == "batch" and world == 1 and not a.no_next:
        t32 = flops / (PEAK_FP32_MFMA_TFLOPS * 1e12)
        with torch.no_grad():
            kernels["fp32_step"] = measure_fp32_step(make_block, coords, B, iters,
                                                     max(t32, t_hbm) + iters * look_bytes / (PEAK_HBM_GBS * 1e9))
    pairs = (world * B if a.mode == "batch" else B) * a.steps
    if a.mode == "batch":
        if (H, W) == (60, 80):
            wl = f"DSEC 480x640 CorrBlock build + {iters} lookups, warm-start, batch {B} per GPU " \
                 f"(BASELINE configs[1]; N>1 = configs[3])"
        elif (H, W) == (32, 32):
            wl = f"MVSEC 256x256 crop CorrBlock build + {iters} lookups, warm-start, batch {B} per GPU " \
                 f"(BASELINE configs[2])"
        else:
            wl = f"{8 * H}x{8 * W} input CorrBlock build + {iters} lookups, warm-start, batch {B} per GPU"
        cfg = {"workload": wl,
               "global_batch": world * B, "fmap": [D, H, W], "levels": 4, "radius": 4,
               "parallelism": f"dp{world} batch-sharded, no collective"}
        if distributed:
            # every rank's own pairs: the sum of its fmap1, gathered after the timed region
            chk = torch.tensor([float(f1.double().sum())], dtype=torch.float64,
                               device="cpu" if single else device)
            allc = [torch.zeros_like(chk) for _ in range(world)]
            dist.all_gather(allc, chk)
            cfg["rank_input_checksums"] = [float(c.item()) for c in allc]
            cfg["rank_seeds"] = [1234 + r for r in range(world)]
    else:
        cfg = {"workload": f"1280x720 CorrBlock build + {iters} lookups, batch {B}, query rows sharded "
                           f"over {world} GPUs (BASELINE configs[4])",
               "global_batch": B, "fmap": [D, H, W], "levels": 4, "radius": 4,
               "parallelism": f"query-row shard x{world}, RCCL all-gather of fmap2 + output slabs"}
        # after the timed region, on every rank: one sharded lookup (the production exchange: RCCL
        # into the persistent chunks + ecorr_rows_assemble) against the unsharded block, bitwise
        with torch.no_grad():
            same = torch.equal(make_block()(coords[0]), eraft_amd.CorrBlock(f1, f2)(coords[0]))
        ok = torch.tensor([1.0 if same else 0.0], dtype=torch.float64, device="cpu" if single else device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        cfg["check_vs_unsharded"] = "bit-exact" if ok.item() == 1.0 else "DIFFERS"
        cfg["row_partition"] = row_partition(H, world)[1]
    res = {
        "metric": METRIC, "value": round(pairs / elapsed, 2), "unit": "pairs/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak" if a.mode == "batch" else "strong",
        "vs_baseline": None, "dtype": "fp32" if mode == "fp32" else "fp32 (f16x3 split MFMA, fp32 accumulate)",
        "data": "synthetic (randn fmaps, coords_grid + smooth warm-start flow)",
        "config": cfg, "roofline": roof, "kernels": kernels,
        "corrblock_frac": round(ideal_s / (elapsed / a.steps), 4),
    }
    if a.mode == "batch" and world == 1 and not a.no_next:
        with torch.no_grad():
            res["next_rows"] = {"lookup_conv1x1_relu": measure_fused_convc1(make_block(), coords, B, H, W, device),
                                "forward_interpolate": measure_forward_interpolate(B, H, W, device),
                                "upsample_flow": measure_upsample(B, H, W, device),
                                "voxel_grid_dsec": measure_voxel(device),
                                "voxel_grid_mvsec": measure_voxel_mvsec(device)}
    if a.mode == "batch" and world == 1 and not a.no_next and not a.no_e2e and (H, W) == (60, 80):
        res["e2e"] = measure_e2e(B, iters, device)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(f1, f2, coords, iters)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if cfg.get("check_vs_unsharded") == "DIFFERS":
        raise SystemExit("row-sharded lookup differs from the unsharded CorrBlock")
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
