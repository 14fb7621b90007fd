#!/usr/bin/env python3
"""Benchmark of the shared-direction PTM fit (BASELINE.json metric).

Metric: Mpix·lights/s of the 6-coefficient PTM fit on a 3840×2160 × 100-light
fp32 stack (BASELINE.json configs[2], the metric's config; it fits one GPU).
One step = one rti_fit_shared launch over the whole stack, inputs resident in
HBM.  With --gpus N (launched by torch.distributed.run) every rank fits its own
2160-row stripe of a G·2160-row image (row-tiled shards, weak scaling) with no
collective in the timed region; --allgather adds the RCCL all-gather that
reassembles the coefficient maps and reports it separately.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--kernel auto]

Rank 0 prints one JSON line.  The CPU baseline (rank 0, N=1) is the oracle's
NumPy restatement (fp64 pinv + fp32 matmul) timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)

CONFIGS = {
    # name: (kind, H, W, lights/evals, channels, basis, description)
    "c2": ("fit", 1080, 1920, 50, 1, "ptm", "ptm6-fit 1920x1080 N=50 fp32 (BASELINE configs[1])"),
    "c3": ("fit", 2160, 3840, 100, 1, "ptm", "ptm6-fit 3840x2160 N=100 fp32 (BASELINE configs[2], metric config)"),
    "c4": ("fit", 2160, 3840, 200, 3, "hsh", "hsh16-fit 3840x2160 RGB N=200 fp32 (BASELINE configs[3])"),
    "c5": ("relight", 2160, 3840, 1000, 1, "ptm",
           "ptm6-relight 3840x2160, 1000 random (lu,lv) streamed one per launch, fp32 out (BASELINE configs[4])"),
    "c6": ("perpixel", 2160, 3840, 100, 1, "ptm",
           "ptm6 per-pixel fit 3840x2160 N=100, light vectors from camera positions in-kernel (reference geometry)"),
    "c7": ("operator", 400, 400, 100, 1, "rbf",
           "linear-RBF interpolation (reference default, SciPy Rbf) of a 400x400 ROI x 100 shared lights on the "
           "100x100 grid -> int32 tables (interpolate_intensities + prepare_images_data)"),
    "c9": ("frame", 2160, 3840, 1000, 1, "ptm",
           "interactive relight frame 3840x2160 (relighting_event): PTM-6 maps at one cursor (lu,lv) -> int32 -> "
           "clip -> V of the HSV ROI -> OpenCV HSV2BGR, one launch per event"),
    "c8": ("rbf_perpixel", 400, 400, 100, 1, "rbf",
           "reference default pipeline: per-pixel linear RBF (own light list per pixel, fp64 LU) of a 400x400 ROI x "
           "100 lights on the 100x100 grid -> int32 tables"),
}
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)


def synth_dirs(n, seed, radius=0.9):
    rng = np.random.default_rng(seed)
    r = radius * np.sqrt(rng.random(n))
    th = 2 * np.pi * rng.random(n)
    return (r * np.cos(th)).astype(np.float32), (r * np.sin(th)).astype(np.float32)


def synth_stack(H, W, N, C, basis, lu, lv, seed, device):
    """I[C, N, H*W] fp32 = clip(round(B·a + N(0,2)), 0, 255) with smooth coefficient fields a."""
    import rti

    g = torch.Generator(device=device).manual_seed(seed)
    k = rti.basis_terms(basis)
    B = torch.as_tensor(rti.design_matrix(lu, lv, basis), device=device, dtype=torch.float32)  # [N, k]
    yy = torch.linspace(0, 1, H, device=device)[:, None]
    xx = torch.linspace(0, 1, W, device=device)[None, :]
    out = torch.empty((C, N, H * W), device=device, dtype=torch.float32)
    for c in range(C):
        a = torch.empty((k, H * W), device=device)
        for j in range(k):
            f1, f2, p1, p2 = (torch.rand(4, generator=g, device=device) * torch.tensor([2.5, 2.5, 6.28, 6.28],
                                                                                      device=device)).tolist()
            s = (torch.sin(2 * np.pi * (f1 + 0.5) * xx + p1) * torch.cos(2 * np.pi * (f2 + 0.5) * yy + p2)).reshape(-1)
            base, amp = (130.0, 70.0) if (basis == "ptm" and j == k - 1) or (basis != "ptm" and j == 0) else (0.0, 50.0)
            a[j] = base + amp * s
        # element-wise accumulation: torch's fp32 GEMM returns wrong values for
        # [n,6] @ [6, 8294400] on this ROCm stack (tools/probe_matmul.py), so no library GEMM here
        Bh = B.cpu().numpy()
        for n in range(N):
            row = torch.randn(H * W, generator=g, device=device) * 2.0
            for j in range(k):
                row.add_(a[j], alpha=float(Bh[n, j]))
            out[c, n] = row.round_().clamp_(0, 255)
        del a
    return out


def load_traffic(workload_key):
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            entry = json.load(f).get(workload_key) or {}
        return entry.get("traffic_bytes_per_launch")
    except (OSError, ValueError):
        return None


def synth_cams(n, seed, H, W):
    """Camera positions on a hemisphere above the image centre (ROI pixel units, analysis.py:228)."""
    rng = np.random.default_rng(seed)
    th = np.arccos(rng.uniform(0.35, 0.95, n))
    ph = rng.uniform(0, 2 * np.pi, n)
    rad = rng.uniform(1.5, 2.5, n) * max(H, W)
    return np.stack([W / 2 + rad * np.sin(th) * np.cos(ph), H / 2 + rad * np.sin(th) * np.sin(ph),
                     rad * np.cos(th)], -1)


def cpu_sample_rate(fn, units, budget_s):
    fn()  # warm-up
    t0 = time.perf_counter()
    reps = 0
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            return units * reps / el / 1e6, reps, el


def cpu_info():
    try:
        from threadpoolctl import threadpool_info
        threads = max([t.get("num_threads", 1) for t in threadpool_info() if t.get("user_api") == "blas"] or [1])
    except Exception:  # pragma: no cover
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    name = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return int(threads), name


class FitWorkload:
    """One step = one rti_fit_shared launch over the rank's whole stack."""

    def __init__(self, args, cfg, rank, dev):
        import rti

        self.rti = rti
        _, H, W, N, C, basis, desc = cfg
        self.H, self.W, self.N, self.C, self.basis, self.desc = H, W, N, C, basis, desc
        self.k = k = rti.basis_terms(basis)
        self.P = P = H * W
        self.args = args
        self.lu, self.lv = synth_dirs(N, seed=2)
        self.I = synth_stack(H, W, N, C, basis, self.lu, self.lv, seed=1000 + rank, device=dev)
        self.in_bytes = 4
        if args.in_dtype != "f32":  # integer-valued 0..255 stacks, as the reference's V channel (analysis.py:219)
            self.I = self.I.to(torch.uint8 if args.in_dtype == "u8" else torch.int32)
            self.in_bytes = 1 if args.in_dtype == "u8" else 4
        self.pinv64 = rti.pinv(self.lu, self.lv, basis)
        self.pinv_dev = torch.as_tensor(self.pinv64.astype(np.float32), device=dev)
        self.coef = torch.empty((C, P, k) if args.layout == "pixel" else (C, k, P), dtype=torch.float32, device=dev)
        self.units = P * N * C
        self.alg_bytes = float(self.in_bytes) * P * N * C + 4.0 * P * k * C  # stack read once + fp32 coefs written
        self.metric = "Mpix*lights/sec PTM fit (4K, 100 lights)" if args.config == "c3" else f"Mpix*lights/sec {desc}"
        self.unit = "Mpix*lights/s"

    def step(self, i):
        self.rti.fit_shared_into(self.pinv_dev, self.I, self.coef, k=self.k, layout=self.args.layout,
                                 kernel=self.args.kernel, nontemporal=self.args.nontemporal)

    def config(self):
        return {"lights": self.N, "channels": self.C, "basis": self.basis, "k": self.k,
                "coef_layout": self.args.layout, "kernel": self.args.kernel, "intensity_dtype": self.args.in_dtype}

    def cpu_baseline(self, budget_s):
        """Oracle restatement: fp64 pinv + fp32 NumPy matmul on light-major rows."""
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import rti_oracle as o

        rows = max(1, self.H // 10)
        sample = self.I[0, :, : rows * self.W].float().cpu().numpy()
        rate, reps, el = cpu_sample_rate(lambda: o.fit_shared_f32(sample, self.pinv64), self.N * rows * self.W,
                                         budget_s)
        threads, name = cpu_info()
        return {"value": round(rate, 1), "unit": self.unit, "cores": threads, "kind": "port",
                "sample": f"oracle fit_shared_f32 (fp64 pinv + fp32 NumPy matmul, channel 0) on {rows}x{self.W} px "
                          f"x {self.N} lights, {reps} reps in {el:.1f}s; {name}"}


class RelightWorkload:
    """One step = one rti_relight launch evaluating ONE (lu, lv) over the 4K coefficient maps (interactive)."""

    def __init__(self, args, cfg, rank, dev):
        import rti

        self.rti = rti
        _, H, W, E, C, basis, desc = cfg
        self.H, self.W, self.E, self.desc, self.basis = H, W, E, desc, basis
        self.k = k = rti.basis_terms(basis)
        self.P = P = H * W
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        self.coef = (torch.rand((P, k), generator=g, device=dev) * 100 - 50).contiguous()
        self.coef[:, k - 1] += 130
        rng = np.random.default_rng(4)
        r = np.sqrt(rng.random(E))
        th = 2 * np.pi * rng.random(E)
        self.luv = torch.as_tensor(np.stack([r * np.cos(th), r * np.sin(th)], -1), device=dev).contiguous()
        self.out = torch.empty((P,), dtype=torch.float32, device=dev)
        self.units = P
        self.alg_bytes = 4.0 * P * k + 4.0 * P  # coefficients read + fp32 image written, per eval
        self.metric = f"Mpix*evals/sec {desc}"
        self.unit = "Mpix*evals/s"
        import ctypes

        self.ctypes = ctypes
        self.lib = rti._lib.lib()
        self.bid = rti.basis_id(basis)

    def step(self, i):
        c = self.ctypes
        e = i % self.E
        st = self.lib.rti_relight(c.c_void_p(self.coef.data_ptr()), self.rti._lib.RTI_F32, self.bid, self.P,
                                  self.rti._lib.RTI_COEF_PIXEL_MAJOR, c.c_void_p(self.luv.data_ptr() + 16 * e), 1,
                                  c.c_void_p(self.out.data_ptr()), self.rti._lib.RTI_F32,
                                  self.rti._lib.RTI_OUT_EVAL_MAJOR,
                                  c.c_void_p(torch.cuda.current_stream().cuda_stream))
        self.rti._lib.check(st, "rti_relight")

    def config(self):
        return {"evals": self.E, "basis": self.basis, "k": self.k, "coef_layout": "pixel", "out": "f32"}

    def cpu_baseline(self, budget_s):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import rti_oracle as o

        rows = max(1, self.H // 10)
        c = self.coef[: rows * self.W].cpu().numpy()
        lu, lv = self.luv[0].cpu().numpy()
        rate, reps, el = cpu_sample_rate(lambda: o.relight(c, self.basis, lu, lv), rows * self.W, budget_s)
        threads, name = cpu_info()
        return {"value": round(rate, 1), "unit": self.unit, "cores": threads, "kind": "port",
                "sample": f"oracle relight (fp64 NumPy) on {rows}x{self.W} px x 1 eval, {reps} reps in {el:.1f}s; "
                          f"{name}"}


class PerPixelWorkload:
    """One step = one rti_fit_perpixel_cam launch (directions from cameras, fp64 normal equations)."""

    def __init__(self, args, cfg, rank, dev):
        import rti

        self.rti = rti
        _, H, W, N, C, basis, desc = cfg
        self.H, self.W, self.N, self.desc = H, W, N, desc
        self.P = P = H * W
        self.cams = synth_cams(N, 6, H, W)
        lu, lv = synth_dirs(N, seed=2)
        self.I = synth_stack(H, W, N, 1, "ptm", lu, lv, seed=1000 + rank, device=dev)[0]  # [N, P]
        self.cams_d = torch.as_tensor(self.cams, device=dev).contiguous()
        self.coef = torch.empty((P, 6), dtype=torch.float32, device=dev)
        self.units = P * N
        self.alg_bytes = 4.0 * P * N + 4.0 * P * 6
        self.metric = f"Mpix*lights/sec {desc}"
        self.unit = "Mpix*lights/s"
        import ctypes

        self.ctypes = ctypes
        self.lib = rti._lib.lib()

    def step(self, i):
        c = self.ctypes
        L = self.rti._lib
        st = self.lib.rti_fit_perpixel_cam(c.c_void_p(self.cams_d.data_ptr()), self.N, c.c_void_p(self.I.data_ptr()),
                                           L.RTI_F32, self.H, self.W, self.P, 0.0, 0.0, -1.0,
                                           c.c_void_p(self.coef.data_ptr()), L.RTI_F32, L.RTI_COEF_PIXEL_MAJOR,
                                           c.c_void_p(torch.cuda.current_stream().cuda_stream))
        L.check(st, "rti_fit_perpixel_cam")

    def config(self):
        return {"lights": self.N, "basis": "ptm", "k": 6, "coef_layout": "pixel", "geometry": "per-pixel cameras"}

    def cpu_baseline(self, budget_s):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import rti_oracle as o

        npx = 4096
        ys, xs = np.divmod(np.arange(npx), self.W)
        lu, lv = o.light_dirs_for_pixels(self.cams, xs, ys)
        I = self.I[:, :npx].cpu().numpy().T
        rate, reps, el = cpu_sample_rate(lambda: o.fit_perpixel(lu, lv, I), npx * self.N, budget_s)
        threads, name = cpu_info()
        return {"value": round(rate, 1), "unit": self.unit, "cores": threads, "kind": "port",
                "sample": f"oracle fit_perpixel (batched fp64 NumPy SVD, reference semantics) on {npx} px x "
                          f"{self.N} lights, {reps} reps in {el:.1f}s; {name}"}


class OperatorWorkload:
    """One step = one rti_apply_operator launch: RBF operator (E = 100x100 grid) over the ROI stack -> int32."""

    def __init__(self, args, cfg, rank, dev):
        import rti

        self.rti = rti
        _, H, W, N, C, basis, desc = cfg
        self.H, self.W, self.N, self.desc = H, W, N, desc
        self.P = P = H * W
        self.lu, self.lv = synth_dirs(N, seed=2)
        self.I = synth_stack(H, W, N, 1, "ptm", self.lu, self.lv, seed=1000 + rank, device=dev)[0]  # [N, P]
        xf = np.around(np.mgrid[-1:1:0.02, -1:1:0.02][1], 2)[0]
        self.qu, self.qv = np.tile(xf, xf.size), np.repeat(xf, xf.size)
        self.E = E = self.qu.size
        self.op64 = rti.rbf_operator(self.lu, self.lv, self.qu, self.qv)  # [N, E] fp64 (host, one-time)
        self.precision = args.op_precision
        self.op = torch.as_tensor(self.op64.astype(np.float32), device=dev).contiguous()
        if self.precision == "split16":
            self.hi, self.lo, self.Kp, self.inv = rti.api.split_operator_f16(self.op64, dev)
        self.out = torch.empty((E, P), dtype=torch.int32, device=dev)
        self.units = P * E
        self.alg_bytes = 4.0 * P * N + 4.0 * P * E  # stack read once + int32 tables written
        self.flops = 2.0 * E * N * P
        self.metric = f"Mpix*evals/sec {desc}"
        self.unit = "Mpix*evals/s"
        import ctypes

        self.ctypes = ctypes
        self.lib = rti._lib.lib()

    def step(self, i):
        c = self.ctypes
        L = self.rti._lib
        stream = c.c_void_p(torch.cuda.current_stream().cuda_stream)
        if self.precision == "split16":
            st = self.lib.rti_apply_operator_f16(c.c_void_p(self.hi.data_ptr()), c.c_void_p(self.lo.data_ptr()),
                                                 self.Kp, self.inv, self.E, self.N, c.c_void_p(self.I.data_ptr()),
                                                 L.RTI_F32, self.P, 1, self.P, self.N * self.P,
                                                 c.c_void_p(self.out.data_ptr()), L.RTI_I32, self.P, self.E * self.P,
                                                 stream)
            L.check(st, "rti_apply_operator_f16")
            return
        st = self.lib.rti_apply_operator(c.c_void_p(self.op.data_ptr()), self.E, self.N, self.E,
                                         c.c_void_p(self.I.data_ptr()), L.RTI_F32, self.P, 1, self.P, self.N * self.P,
                                         c.c_void_p(self.out.data_ptr()), L.RTI_I32, self.P, self.E * self.P, stream)
        L.check(st, "rti_apply_operator")

    def config(self):
        return {"lights": self.N, "evals": self.E, "basis": "rbf-linear", "out": "int32 tables [E][P]",
                "operator_precision": self.precision}

    def roofline(self, kernel_ms):
        ach = self.flops / (kernel_ms * 1e-3) / 1e12
        if self.precision == "split16":
            # two f16 MFMA products per multiply-add put the compute at 2 x 3.2e11 x 1.12 flop per launch
            # (~0.3 ms at the dense f16 peak), so the E x P int32 table writes (6.4 GB) bound it: HBM roofline
            gbs = self.alg_bytes / (kernel_ms * 1e-3) / 1e9
            return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None, "kernel_ms": round(kernel_ms, 4),
                    "alg_bytes_per_launch": self.alg_bytes, "alg_flops_per_launch": self.flops,
                    "mfma_f16_TFLOPs_issued": round(2 * self.flops * (self.Kp / self.N) / (kernel_ms * 1e-3) / 1e12, 1),
                    "mfma_f16_peak": 2516.6}
        return {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / MFMA_F32_PEAK_TFLOPS, 4), "traffic": None, "kernel_ms": round(kernel_ms, 4),
                "alg_flops_per_launch": self.flops, "alg_bytes_per_launch": self.alg_bytes,
                "hbm_GBps": round(self.alg_bytes / (kernel_ms * 1e-3) / 1e9, 1)}

    def cpu_baseline(self, budget_s):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        npx = 256
        I = self.I[:, :npx].cpu().numpy().astype(np.float64)
        op = self.op64
        rate, reps, el = cpu_sample_rate(lambda: (op.T @ I).astype(np.int32), npx * self.E, budget_s)
        threads, name = cpu_info()
        return {"value": round(rate, 1), "unit": self.unit, "cores": threads, "kind": "port",
                "sample": f"NumPy fp64 operator product (the SciPy-Rbf-equivalent grid) on {npx} px x {self.E} "
                          f"evals, {reps} reps in {el:.1f}s; {name}"}


class RbfPerPixelWorkload:
    """One step = one rti_rbf_perpixel launch over the ROI: per-pixel fp64 solve + 10^4 evaluations."""

    def __init__(self, args, cfg, rank, dev):
        import rti

        self.rti = rti
        _, H, W, N, C, basis, desc = cfg
        self.H, self.W, self.N, self.desc = H, W, N, desc
        self.P = P = H * W
        cams = synth_cams(N, 6, H, W)
        ys, xs = np.divmod(np.arange(P), W)
        dx = cams[None, :, 0] - xs[:, None]
        dy = cams[None, :, 1] - ys[:, None]
        nrm = np.sqrt(dx * dx + dy * dy + cams[None, :, 2] ** 2)
        self.lu_h = (dx / nrm).astype(np.float32)
        self.lv_h = (dy / nrm).astype(np.float32)
        self.lu = torch.as_tensor(self.lu_h, device=dev)
        self.lv = torch.as_tensor(self.lv_h, device=dev)
        rng = np.random.default_rng(7 + rank)
        self.I_h = rng.integers(0, 256, (P, N)).astype(np.int32)
        self.I = torch.as_tensor(self.I_h, device=dev)
        xf = np.around(np.mgrid[-1:1:0.02, -1:1:0.02][1], 2)[0]
        self.qu, self.qv = np.tile(xf, xf.size), np.repeat(xf, xf.size)
        self.E = E = self.qu.size
        self.luv = torch.as_tensor(np.stack([self.qu, self.qv], -1), device=dev).contiguous()
        self.out = torch.empty((E, P), dtype=torch.int32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.units = P * E
        self.alg_bytes = 12.0 * P * N + 4.0 * P * E
        self.flops = P * (2.0 / 3.0 * N ** 3 + 5.0 * N * N + 8.0 * N * E)  # LU + A build + evaluation (fp64)
        self.metric = f"Mpix*evals/sec {desc}"
        self.unit = "Mpix*evals/s"
        import ctypes

        self.ctypes = ctypes
        self.lib = rti._lib.lib()

    def step(self, i):
        c = self.ctypes
        L = self.rti._lib
        st = self.lib.rti_rbf_perpixel(c.c_void_p(self.lu.data_ptr()), c.c_void_p(self.lv.data_ptr()),
                                       c.c_void_p(self.I.data_ptr()), L.RTI_I32, self.N, self.P,
                                       c.c_void_p(self.luv.data_ptr()), self.E, c.c_void_p(self.out.data_ptr()),
                                       L.RTI_I32, L.RTI_OUT_EVAL_MAJOR, c.c_void_p(self.status.data_ptr()),
                                       c.c_void_p(torch.cuda.current_stream().cuda_stream))
        L.check(st, "rti_rbf_perpixel")

    def config(self):
        return {"lights": self.N, "evals": self.E, "basis": "rbf-linear per-pixel", "out": "int32 tables [E][P]"}

    def roofline(self, kernel_ms):
        ach = self.flops / (kernel_ms * 1e-3) / 1e12
        return {"bound": "fp64-valu", "achieved": round(ach, 2), "peak": 78.6, "unit": "TFLOP/s",
                "frac": round(ach / 78.6, 4), "traffic": None, "kernel_ms": round(kernel_ms, 4),
                "alg_flops_per_launch": self.flops, "alg_bytes_per_launch": self.alg_bytes}

    def cpu_baseline(self, budget_s):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import rti_oracle as o

        npx = 16
        def run():
            for p in range(npx):
                o.rbf_linear(self.lu_h[p], self.lv_h[p], self.I_h[p], self.qu, self.qv)
        rate, reps, el = cpu_sample_rate(run, npx * self.E, budget_s)
        threads, name = cpu_info()
        return {"value": round(rate, 3), "unit": self.unit, "cores": threads, "kind": "port",
                "sample": f"oracle rbf_linear (SciPy-equivalent fp64 solve + cdist eval) on {npx} px x {self.E} "
                          f"evals, {reps} reps in {el:.1f}s; {name}"}


class FrameWorkload(RelightWorkload):
    """One step = one rti_relight_frame launch: the image relighting_event shows for one cursor position
    (interactive_relighting.py:31-38), from device-resident coefficient maps and HSV ROI."""

    def __init__(self, args, cfg, rank, dev):
        super().__init__(args, cfg, rank, dev)
        g = torch.Generator(device=dev).manual_seed(2000 + rank)
        self.hsv = torch.randint(0, 256, (self.P, 3), generator=g, device=dev, dtype=torch.uint8)
        self.bgr = torch.empty((self.P, 3), dtype=torch.uint8, device=dev)
        self.luv_host = self.luv.cpu().numpy()
        self.alg_bytes = 4.0 * self.P * self.k + 3.0 * self.P + 3.0 * self.P  # coefficients + HSV in, BGR out

    def step(self, i):
        c = self.ctypes
        lu, lv = self.luv_host[i % self.E]
        st = self.lib.rti_relight_frame(c.c_void_p(self.coef.data_ptr()), self.rti._lib.RTI_F32, self.bid,
                                        self.rti._lib.RTI_COEF_PIXEL_MAJOR, self.P, float(lu), float(lv),
                                        c.c_void_p(self.hsv.data_ptr()), c.c_void_p(self.bgr.data_ptr()),
                                        c.c_void_p(torch.cuda.current_stream().cuda_stream))
        self.rti._lib.check(st, "rti_relight_frame")

    def config(self):
        return {"events": self.E, "basis": self.basis, "k": self.k, "coef_layout": "pixel",
                "out": "uint8 BGR [P][3]"}

    def cpu_baseline(self, budget_s):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import rti_oracle as o

        rows = max(1, self.H // 10)
        c = self.coef[: rows * self.W].cpu().numpy()
        hsv = self.hsv[: rows * self.W].cpu().numpy().reshape(rows, self.W, 3)
        lu, lv = self.luv_host[0]

        def one():
            v = o.relight(c, self.basis, lu, lv).reshape(rows, self.W)
            return o.relighting_event_image(np.trunc(v).astype(np.int32), hsv)

        rate, reps, el = cpu_sample_rate(one, rows * self.W, budget_s)
        threads, name = cpu_info()
        return {"value": round(rate, 1), "unit": self.unit, "cores": threads, "kind": "port",
                "sample": f"oracle relight + clip + HSV2BGR (NumPy) on {rows}x{self.W} px x 1 event, {reps} reps in "
                          f"{el:.1f}s; {name}"}


WORKLOADS = {"fit": FitWorkload, "relight": RelightWorkload, "perpixel": PerPixelWorkload, "frame": FrameWorkload,
             "operator": OperatorWorkload, "rbf_perpixel": RbfPerPixelWorkload}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 20 (fit) / 1000 (relight) / 10 (per-pixel)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--kernel", default="auto", choices=["auto", "valu", "mfma"])
    ap.add_argument("--layout", default="pixel", choices=["pixel", "planar"])
    ap.add_argument("--nontemporal", action="store_true")
    ap.add_argument("--in-dtype", default="f32", choices=["f32", "u8", "i32"],
                    help="intensity stack type for fit configs (BASELINE's metric is fp32)")
    ap.add_argument("--op-precision", default="split16", choices=["split16", "fp32"],
                    help="c7: operator as two fp16 halves on f16 MFMA (default) or fp32 on f32 MFMA")
    ap.add_argument("--allgather", action="store_true", help="also time the RCCL all-gather of the maps")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for real runs; gloo lets ranks share one GPU in rehearsals")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    kind = cfg[0]
    if args.steps is None:
        args.steps = {"fit": 20, "relight": 1000, "frame": 1000, "perpixel": 10, "operator": 10, "rbf_perpixel": 3}[kind]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    import rti

    rti.load()
    wl = WORKLOADS[kind](args, cfg, rank, dev)
    torch.cuda.synchronize(dev)

    for i in range(args.warmup):
        wl.step(i)
    torch.cuda.synchronize(dev)

    stream = torch.cuda.current_stream(dev)
    # timed region: exactly K steps between barrier + synchronize, nothing else enqueued
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        wl.step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # kernel duration for the roofline: HIP events around each launch, on the launch stream,
    # in a separate pass so the events do not add gaps to the timed region
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for i in range(args.steps):
        ev[i][0].record(stream)
        wl.step(i)
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])

    gather_ms = e2e_ms = None
    if args.allgather and world > 1 and kind == "fit":
        from rti.parallel import gather_rows

        H, W, k = wl.H, wl.W, wl.k
        local_map = wl.coef[0].reshape(H, W, k) if args.layout == "pixel" else wl.coef[0].reshape(k, H, W)
        for _ in range(2):
            gather_rows(local_map, H * world)
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(5):
            gather_rows(local_map, H * world)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) / 5 * 1e3
        # end to end: the row-chunked fit with each chunk's all-gather overlapped with the next fit
        from rti.parallel import fit_rowtiled_overlapped

        Irows = wl.I[0].reshape(wl.N, H, W)
        for _ in range(2):
            fit_rowtiled_overlapped(Irows, wl.lu, wl.lv, H * world, basis=wl.basis, chunks=4)
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(5):
            fit_rowtiled_overlapped(Irows, wl.lu, wl.lv, H * world, basis=wl.basis, chunks=4)
        torch.cuda.synchronize(dev)
        e2e_ms = (time.perf_counter() - g0) / 5 * 1e3

    value = world * wl.units * args.steps / elapsed / 1e6
    achieved = wl.alg_bytes / (kernel_ms * 1e-3) / 1e9
    workload_key = f"{args.config}-{args.kernel}-{args.layout}" + ("" if args.in_dtype == "f32" else f"-{args.in_dtype}")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = wl.cpu_baseline(args.cpu_budget)
    if rank == 0:
        conf = {"workload": wl.desc, "H_per_rank": wl.H, "W": wl.W}
        conf.update(wl.config())
        conf["parallelism"] = f"row-stripes x{world} (one {wl.H}-row stripe per GPU)"
        line = {
            "metric": wl.metric,
            "value": round(value, 1),
            "unit": wl.unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"perpixel": "f32 in / f64 solve", "operator": ("f32 operator as 2 x f16 (f16 MFMA, f32 accumulate) -> int32"
                                                       if args.op_precision == "split16" else "f32 (MFMA) -> int32"),
                      "rbf_perpixel": "f64 -> int32", "frame": "f32 eval -> u8 BGR"}.get(kind, "f32" if args.in_dtype == "f32"
                                                          else f"{args.in_dtype} in / f32 compute"),
            "data": "synthetic (seeded smooth PTM/HSH coefficient fields + N(0,2) noise, rounded to 0..255, fp32)",
            "config": conf,
            "roofline": wl.roofline(kernel_ms) if hasattr(wl, "roofline") else {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(workload_key),
                "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": wl.alg_bytes},
            "cpu_baseline": cpu,
        }
        if gather_ms is not None:
            line["allgather_ms"] = round(gather_ms, 3)
            line["fit_allgather_overlapped_ms"] = round(e2e_ms, 3)  # 4 row chunks, gather(c) || fit(c+1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
