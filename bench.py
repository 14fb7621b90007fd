#!/usr/bin/env python3
"""Benchmark of the shared-direction PTM fit (BASELINE.json metric) and the other §8 rows.

Metric: Mpix·lights/s of the 6-coefficient PTM fit on a 3840×2160 × 100-light fp32 stack
(BASELINE.json configs[2], "at 1/2/4/8 GPU").  One step = one rti_fit_shared call per rank over that
rank's row block (AUTO issues it as launches_per_step launch generations), inputs resident in HBM.

Multi-GPU: one process per GPU.  ``--gpus N`` without WORLD_SIZE in the
environment re-launches this script under ``torch.distributed.run`` with N ranks (before the
parent touches the GPU); the driver's own torchrun launch is used as is.  Default = STRONG
scaling: rank r fits rows row_range(H, G, r) (2160/G rows of the same 4K image) with the
replicated k×N pseudo-inverse and no collective in the timed region; value = all pixel·lights of
the image ÷ the max-over-ranks time.  ``--weak`` gives every rank a whole H-row image instead.
The RCCL all-gather that reassembles the maps (the north_star's only collective) is timed
separately (``allgather_ms``), and so is the row-chunked fit with each chunk's all-gather
overlapped with the next chunk's fit (``fit_allgather_overlapped_ms``).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--weak]

Rank 0 prints one JSON line.  It carries ``roofline`` (kernel time = median of 50 HIP-event
windows on the launch stream after 10 warm-ups, each window ≥ 1 ms of back-to-back launches), an in-run ``parity`` check of sampled outputs
against the CPU oracle (BASELINE.md plan step 5) and ``cpu_baseline`` (rank 0, N = 1: the
oracle's NumPy restatement on a bounded sample, at the affinity thread count and at 1 thread).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6

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
    "c8": ("rbf_perpixel", 400, 400, 100, 1, "rbf",
           "reference default pipeline: per-pixel linear RBF (own light list per pixel, fp64 LU) of a 400x400 ROI x "
           "100 lights on the 100x100 grid -> int32 tables"),
    "c8n200": ("rbf_perpixel", 400, 400, 200, 1, "rbf",
               "reference default pipeline at N=200 (SURVEY §6): per-pixel linear RBF of a 400x400 ROI x 200 lights "
               "on the 100x100 grid -> int32 tables"),
    "c8n400": ("rbf_perpixel", 400, 400, 400, 1, "rbf",
               "reference default pipeline above 256 lights (a 100 s capture: N = frames/8, analysis.py:120,152): "
               "per-pixel linear RBF of a 400x400 ROI x 400 lights (blocked fp64 Cholesky) on the 100x100 grid -> "
               "int32 tables"),
    "c9": ("frame", 2160, 3840, 1000, 1, "ptm",
           "interactive relight frame 3840x2160 (relighting_event): PTM-6 maps at one cursor (lu,lv) -> int32 -> "
           "clip -> V of the HSV ROI -> OpenCV HSV2BGR, one launch per event"),
    "c10": ("fit_residual", 2160, 3840, 100, 1, "ptm",
            "ptm6-fit + per-pixel residuals in ONE pass, 3840x2160 N=100 fp32 (north_star residuals)"),
}
DEFAULT_STEPS = {"fit": 20, "fit_residual": 20, "relight": 1000, "frame": 1000, "perpixel": 10, "operator": 10,
                 "rbf_perpixel": 3}


# ---- launcher ---------------------------------------------------------------------------------

def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def maybe_spawn(args):
    """--gpus N > 1 outside a torchrun launch: start N fresh ranks under torch.distributed.run and
    exit with their status.  Runs before anything in this process touches the GPU."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.run(cmd, env=env).returncode)


class Ctx:
    """This rank's share of the image: rows [r0, r1) of an H-row image."""

    def __init__(self, args, H, rank, world, dev):
        from rti.parallel import row_range

        self.rank, self.world, self.dev, self.weak = rank, world, dev, args.weak
        if args.weak:  # every rank a whole H-row image stacked below the others
            self.H, self.r0, self.r1 = H * world, rank * H, (rank + 1) * H
        else:
            self.H = H
            self.r0, self.r1 = row_range(H, world, rank)
        self.h = self.r1 - self.r0


# ---- synthetic inputs -------------------------------------------------------------------------

def synth_dirs(n, seed, radius=0.9):
    rng = np.random.default_rng(seed)
    r = radius * np.sqrt(rng.random(n))
    th = 2 * np.pi * rng.random(n)
    return (r * np.cos(th)).astype(np.float32), (r * np.sin(th)).astype(np.float32)


def synth_stack(H, W, N, C, basis, lu, lv, seed, device, rows=None):
    """Rows [r0, r1) of I[C, N, H*W] fp32 = clip(round(B·a + N(0,2)), 0, 255) with smooth coefficient
    fields a(y, x) of the whole H×W image (identical on every rank; the noise is per row block)."""
    import torch

    import rti

    r0, r1 = rows or (0, H)
    h = r1 - r0
    g = torch.Generator(device=device).manual_seed(seed)
    gn = torch.Generator(device=device).manual_seed(seed * 7919 + r0)
    k = rti.basis_terms(basis)
    B = rti.design_matrix(lu, lv, basis)  # [N, k] host fp64
    yy = torch.linspace(0, 1, H, device=device)[r0:r1, None]
    xx = torch.linspace(0, 1, W, device=device)[None, :]
    out = torch.empty((C, N, h * W), device=device, dtype=torch.float32)
    for c in range(C):
        a = torch.empty((k, h * W), device=device)
        for j in range(k):
            f1, f2, p1, p2 = (torch.rand(4, generator=g, device=device) * torch.tensor([2.5, 2.5, 6.28, 6.28],
                                                                                      device=device)).tolist()
            s = (torch.sin(2 * np.pi * (f1 + 0.5) * xx + p1) * torch.cos(2 * np.pi * (f2 + 0.5) * yy + p2)).reshape(-1)
            base, amp = (130.0, 70.0) if (basis == "ptm" and j == k - 1) or (basis != "ptm" and j == 0) else (0.0, 50.0)
            a[j] = base + amp * s
        # element-wise accumulation: torch's fp32 GEMM returns wrong values for
        # [n,6] @ [6, 8294400] on this ROCm stack (tools/probe_matmul.py), so no library GEMM here
        for n in range(N):
            row = torch.randn(h * W, generator=gn, device=device) * 2.0
            for j in range(k):
                row.add_(a[j], alpha=float(B[n, j]))
            out[c, n] = row.round_().clamp_(0, 255)
        del a
    return out


def synth_cams(n, seed, H, W):
    """Camera positions on a hemisphere above the image centre (ROI pixel units, analysis.py:228)."""
    rng = np.random.default_rng(seed)
    th = np.arccos(rng.uniform(0.35, 0.95, n))
    ph = rng.uniform(0, 2 * np.pi, n)
    rad = rng.uniform(1.5, 2.5, n) * max(H, W)
    return np.stack([W / 2 + rad * np.sin(th) * np.cos(ph), H / 2 + rad * np.sin(th) * np.sin(ph),
                     rad * np.cos(th)], -1)


# source files that define each profiled kernel (and what it includes); the PMC traffic recorded for a kernel
# is reported only while these files are byte-identical to the ones the counters were taken on
KERNEL_SOURCES = {
    "fit_shared_valu": ["rti_fit.hip"], "fit_shared_tile": ["rti_fit.hip"], "fit_shared_mfma": ["rti_fit.hip"],
    "fit_q8": ["rti_fit_q8.hip", "rti_q8.h"], "fit_pm": ["rti_fit_pm.hip"], "fit_h16": ["rti_fit_h16.hip"], "fit_shared_residual_k": ["rti_fitres.hip"],
    "fit_residual_k": ["rti_residual.hip"], "relight_eval": ["rti_relight.hip", "rti_convert.h"],
    "relight_frame": ["rti_relight.hip", "rti_convert.h"], "fit_perpixel_cam": ["rti_perpixel.hip"],
    "apply_op": ["rti_operator.hip"], "rbf_": ["rti_rbf.hip"],
}
COMMON_SOURCES = ["rti_internal.h", "rti_basis.h"]


def kernel_sources(kernel_regex):
    for root, files in KERNEL_SOURCES.items():
        if kernel_regex.startswith(root) or root.startswith(kernel_regex):
            return [f"smartphone-based-rti_amd/csrc/{f}" for f in files + COMMON_SOURCES]
    return None


def sources_sha16(files):
    import hashlib

    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def load_traffic(workload_key, family=None):
    """PMC bytes per step for this workload from profiles/traffic.json, with its provenance: reported only when
    the kernel source files the counters were taken on (entry['sources'], hashed as entry['src_sha16']) are
    unchanged and, when the caller names the kernel family it launched (e.g. "fit_h16"), the profiled kernel
    symbol is of that family — otherwise traffic None and traffic_source.stale = true."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            entry = json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None, None
    if not entry:
        return None, None
    src = {"key": workload_key, "kernel": entry.get("kernel_symbol"), "commit": entry.get("commit"),
           "src_sha16": entry.get("src_sha16")}
    files = entry.get("sources")
    try:
        now = sources_sha16(files) if files else None
    except OSError:
        now = None
    src["stale"] = not (files and now == entry.get("src_sha16")) or \
        bool(family and family not in (entry.get("kernel_symbol") or ""))
    if src["stale"]:
        return None, src
    # per step: launch generations split one step into launches_per_step launches
    return entry.get("traffic_bytes_per_step", entry.get("traffic_bytes_per_launch")), src


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rti_oracle

    return rti_oracle


def sample_idx(P, n, seed):
    rng = np.random.default_rng(seed)
    if P <= n:
        return np.arange(P)
    return np.sort(rng.choice(P, n, replace=False))


def torch_idx(idx, device):
    import torch

    return torch.as_tensor(idx, device=device)


def coef_parity(got, ref):
    """max over pixels of max_k |c - c_ref| / max(max_k |c_ref|, 1e-30)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.maximum(np.abs(ref).max(-1, keepdims=True), 1e-30)
    return float((np.abs(got - ref) / scale).max())


def int_table_parity(got, ref_float):
    """int32 outputs (C truncation): exact match except where the fp64 value sits within 1e-4 of an
    integer (the truncation may then fall either way)."""
    ref_i = np.trunc(ref_float).astype(np.int64)
    diff = np.asarray(got, np.int64) != ref_i
    near = np.abs(ref_float - np.round(ref_float)) < 1e-4
    return {"checked": int(diff.size), "mismatch": int(diff.sum()), "mismatch_not_near_integer": int((diff & ~near).sum()),
            "ok": bool(not (diff & ~near).any())}


# ---- workloads --------------------------------------------------------------------------------

class Workload:
    """Subclasses set units (this rank's work per step), total_units, alg_bytes (per launch),
    metric, unit, desc and implement step(i), config(), parity() and cpu_fn()."""

    dtype = "f32"

    launches = 1  # kernel launches per step (fits: rti_last_launch_count after a step, launch generations)

    def roofline(self, kernel_ms):
        """achieved = algorithmic bytes of one step / the step's kernel time (event-timed on the launch
        stream; with L > 1 launch generations per step that time includes the L - 1 launch boundaries,
        and rocprofv3's per-launch average x L is the gap-free figure)."""
        gbs = self.alg_bytes / (kernel_ms * 1e-3) / 1e9
        L = int(self.launches)
        traffic, tsrc = self.traffic_entry()
        return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                "kernel_ms": round(kernel_ms, 4),
                "alg_bytes_per_launch": self.alg_bytes / L, "alg_bytes_per_step": self.alg_bytes,
                "launches_per_step": L, "kernel_ms_per_launch": round(kernel_ms / L, 5)}

    def traffic(self):
        return None

    def traffic_entry(self):
        """(PMC traffic bytes per step or None, its provenance or None)."""
        t = self.traffic()
        return t if isinstance(t, tuple) else (t, None)


class FitWorkload(Workload):
    """One step = one rti_fit_shared call (launches_per_step launches) over this rank's row block."""

    def __init__(self, args, cfg, ctx):
        import torch

        import rti

        self.rti, self.args, self.ctx = rti, args, ctx
        _, H, W, N, C, basis, desc = cfg
        self.W, self.N, self.C, self.basis, self.desc = W, N, C, basis, desc
        self.k = k = rti.basis_terms(basis)
        self.P = P = ctx.h * W
        dev = ctx.dev
        self.lu, self.lv = synth_dirs(N, seed=2)
        self.I = synth_stack(ctx.H, W, N, C, basis, self.lu, self.lv, seed=1000, device=dev, rows=(ctx.r0, ctx.r1))
        self.in_bytes = 4
        if args.in_dtype != "f32":  # integer-valued 0..255 stacks, as the reference's V channel (analysis.py:219)
            self.I = self.I.to(torch.uint8 if args.in_dtype == "u8" else torch.int32)
            self.in_bytes = 1 if args.in_dtype == "u8" else 4
        self.stack = getattr(args, "stack", "light")
        if self.stack == "pixel":  # the reference's own (R, R, N) layout (analysis.py:217-219): I[c][p][n]
            self.I = self.I.transpose(1, 2).contiguous()
        self.pinv64 = rti.pinv(self.lu, self.lv, basis)
        self.pinv_dev = torch.as_tensor(self.pinv64.astype(np.float32), device=dev)
        self.coef = torch.empty((C, P, k) if args.layout == "pixel" else (C, k, P), dtype=torch.float32, device=dev)
        self.units = P * N * C
        self.total_units = ctx.H * W * N * C
        self.alg_bytes = float(self.in_bytes) * P * N * C + 4.0 * P * k * C  # stack read once + fp32 coefs written
        self.metric = ("Mpix*lights/sec PTM fit (4K, 100 lights)" if args.config == "c3"
                       else f"Mpix*lights/sec {desc}")
        self.unit = "Mpix*lights/s"
        self.dtype = "f32" if args.in_dtype == "f32" else f"{args.in_dtype} in / f32 compute"
        L = rti._lib
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        # 8-bit stacks: rti.fit's AUTO path, the split-fp16 fit on the fp16 matrix cores (rti_fit_h16.hip), or
        # with --kernel q8 the int8 fixed-point form (rti_fit_q8.hip)
        mk = "h16" if args.kernel == "auto" else args.kernel
        self.q8 = self.stack == "light" and mk in ("h16", "q8") and rti.api.q8_supported(self.I, k, N, P, mk)
        self.u8_kernel = mk if self.q8 else None
        if self.q8:
            if mk == "h16":
                self.op_dev = torch.as_tensor(rti.h16_operator(self.pinv64), device=dev)
                fn, fname = L.lib().rti_fit_shared_h16, "rti_fit_shared_h16"
            else:
                self.op_dev = torch.as_tensor(rti.q8_operator(self.pinv64), device=dev)
                fn, fname = L.lib().rti_fit_shared_q8, "rti_fit_shared_q8"
            cargs = (ctypes.c_void_p(self.op_dev.data_ptr()), k, N, ctypes.c_void_p(self.I.data_ptr()), P, C, P, N * P,
                     ctypes.c_void_p(self.coef.data_ptr()), rti.api._layout_id(args.layout), P * k, 0, stream)
        elif self.stack == "pixel":  # rti_fit_shared_pm: pixel stride N, channel stride P·N
            fn, fname = L.lib().rti_fit_shared_pm, "rti_fit_shared_pm"
            cargs = (ctypes.c_void_p(self.pinv_dev.data_ptr()), k, N, ctypes.c_void_p(self.I.data_ptr()),
                     rti.api._IN_DTYPES[self.I.dtype], P, C, N, P * N, ctypes.c_void_p(self.coef.data_ptr()),
                     rti.api._layout_id(args.layout), P * k, rti.api._KERNELS[args.kernel], stream)
            self.pm_plan = int(L.lib().rti_fit_shared_pm_plan(k, N, rti.api._IN_DTYPES[self.I.dtype], P, C, N, P * N,
                                                              rti.api._KERNELS[args.kernel]))
        else:
            kern = rti.api._KERNELS[args.kernel] | (L.RTI_KERNEL_NONTEMPORAL if args.nontemporal else 0)
            fn, fname = L.lib().rti_fit_shared, "rti_fit_shared"
            cargs = (ctypes.c_void_p(self.pinv_dev.data_ptr()), k, N, ctypes.c_void_p(self.I.data_ptr()),
                     rti.api._IN_DTYPES[self.I.dtype], P, C, P, N * P, ctypes.c_void_p(self.coef.data_ptr()),
                     rti.api._layout_id(args.layout), P * k, kern, stream)

        def step(i):
            st = fn(*cargs)
            if st:
                L.check(st, fname)

        self.step = step
        step(0)
        self.launches = int(L.lib().rti_last_launch_count())
        if self.u8_kernel == "q8":
            self.dtype = "u8 in / int8 MFMA on a 4-digit 27-bit fixed-point operator, exact int32 sums / f32 out"
        elif self.u8_kernel == "h16":
            self.dtype = "u8 in / fp16 MFMA on a split-fp16 (22-bit) operator, fp32 sums / f32 out"

    def traffic(self):
        if self.ctx.world != 1 or self.ctx.weak:
            return None  # the PMC figures in profiles/traffic.json are for the whole image
        a = self.args
        key = f"{a.config}-{a.kernel}-{a.layout}" + ("" if a.in_dtype == "f32" else f"-{a.in_dtype}") + \
            ("-pm" if self.stack == "pixel" else "")
        fam = f"fit_{self.u8_kernel}" if self.u8_kernel else ("fit_pm" if self.stack == "pixel" else None)
        return load_traffic(key, fam)

    def config(self):
        cfg = {"lights": self.N, "channels": self.C, "basis": self.basis, "k": self.k,
               "coef_layout": self.args.layout, "kernel": self.u8_kernel or self.args.kernel,
               "intensity_dtype": self.args.in_dtype, "stack_layout": self.stack}
        if self.stack == "pixel":
            form = {1: "valu generations (one pixel per lane, packed FMA, coefficients parked until the launch's end)",
                    2: "mfma stream", 3: "mfma block", 4: "direct (stack straight into MFMA operands)"}
            cfg["pm_plan"] = {"form": form.get(self.pm_plan // 100000000), "waves_per_cu": self.pm_plan % 1000,
                              "kib_ring_or_px_block": self.pm_plan % 100000000 // 1000} \
                if self.pm_plan else "one lane per pixel"
        return cfg

    def stack_cols(self, c, idx):
        """[N, len(idx)] intensities of channel c at pixels idx, whatever the stack layout."""
        return self.I[c][idx, :].T if self.stack == "pixel" else self.I[c][:, idx]

    def coef_pk(self, c):
        cc = self.coef[c]
        return cc if self.args.layout == "pixel" else cc.T

    def parity(self):
        o = oracle()
        idx = sample_idx(self.P, 4096, 11 + self.ctx.rank)
        worst = 0.0
        for c in sorted({0, self.C - 1}):
            I = self.stack_cols(c, torch_idx(idx, self.I.device)).float().cpu().numpy()
            ref = o.fit_shared(I, self.pinv64)
            got = self.coef_pk(c)[idx].cpu().numpy()
            worst = max(worst, coef_parity(got, ref))
        return {"max_rel": worst, "tol": 1e-4, "ok": bool(worst <= 1e-4), "checked_px": int(len(idx)),
                "vs": "oracle fit_shared (fp64 pinv, fp64 contraction)"}

    def cpu_fn(self):
        o = oracle()
        rows = max(1, min(self.ctx.h, 216))
        sample = (self.I[0, : rows * self.W, :].T if self.stack == "pixel" else self.I[0, :, : rows * self.W]).float()
        sample = np.ascontiguousarray(sample.cpu().numpy())
        return (lambda: o.fit_shared_f32(sample, self.pinv64), self.N * rows * self.W,
                f"oracle fit_shared_f32 (fp64 pinv + fp32 NumPy matmul, channel 0) on {rows}x{self.W} px x {self.N} "
                f"lights")

    def cpu_ref_fn(self):
        """The reference's OWN least-squares path, not the port: every pixel builds its N x k design matrix
        from its light list (analysis.py:280-291, float32 monomials with powf squares) and solves it with a
        full fp64 SVD and no rcond (analysis.py:293-298), as interpolate_intensities calls it per pixel
        (analysis.py:350-359); here batched (oracle.fit_perpixel) on the first rows of the same stack with the
        shared directions broadcast to every pixel."""
        o = oracle()
        rows = max(1, min(self.ctx.h, 8))
        npx = rows * self.W
        sample = (self.I[0, :npx, :] if self.stack == "pixel" else self.I[0, :, :npx].T).float()
        sample = np.ascontiguousarray(sample.cpu().numpy())
        lu = np.broadcast_to(self.lu[None, :], (npx, self.N))
        lv = np.broadcast_to(self.lv[None, :], (npx, self.N))
        return (lambda: o.fit_perpixel(lu, lv, sample, self.basis), self.N * npx,
                f"oracle fit_perpixel (per-pixel design matrix + batched fp64 NumPy SVD, no rcond: the reference's "
                f"analysis.py:280-298 semantics, channel 0) on {rows}x{self.W} px x {self.N} lights")


class FitResidualWorkload(FitWorkload):
    """One step = one rti_fit_shared_residual_svd call (what rti.fit_with_residual runs): coefficients +
    per-pixel RMS residuals + per-workgroup residual energy in one pass over the stack (fp64 accumulation of
    Uᵀ I and ‖I‖², the reference's SVD solve)."""

    def __init__(self, args, cfg, ctx):
        import torch

        super().__init__(args, cfg, ctx)
        rti, L = self.rti, self.rti._lib
        k, N, C, P = self.k, self.N, self.C, self.P
        dev = ctx.dev
        U, Wf = rti.lsq_factors(self.lu, self.lv, self.basis)
        self.A64 = rti.design_matrix(self.lu, self.lv, self.basis)
        self.A_dev = torch.as_tensor(U, device=dev).contiguous()
        self.ginv_dev = torch.as_tensor(Wf, device=dev).contiguous()
        self.res = torch.empty((C, P), dtype=torch.float32, device=dev)
        nb = int(L.lib().rti_fit_shared_residual_blocks(P))
        self.partial = torch.zeros((C, nb), dtype=torch.float64, device=dev)
        self.alg_bytes += 4.0 * P * C  # + fp32 residual map
        self.metric = f"Mpix*lights/sec {self.desc}"
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        fn = L.lib().rti_fit_shared_residual_svd
        cargs = (ctypes.c_void_p(self.A_dev.data_ptr()), ctypes.c_void_p(self.ginv_dev.data_ptr()), k, N,
                 ctypes.c_void_p(self.I.data_ptr()), rti.api._IN_DTYPES[self.I.dtype], P, C, P, N * P,
                 ctypes.c_void_p(self.coef.data_ptr()), rti.api._layout_id(args.layout), P * k,
                 ctypes.c_void_p(self.res.data_ptr()), ctypes.c_void_p(self.partial.data_ptr()), 0, stream)

        def step(i):
            st = fn(*cargs)
            if st:
                L.check(st, "rti_fit_shared_residual_svd")

        self.step = step
        step(0)
        self.launches = int(L.lib().rti_last_launch_count())
        self.dtype = "f32 in / f64 accumulate / f32 out"

    def traffic(self):
        if self.ctx.world != 1 or self.ctx.weak:
            return None
        return load_traffic(self.args.config)

    def parity(self):
        o = oracle()
        idx = sample_idx(self.P, 4096, 13 + self.ctx.rank)
        worst = worst_r = 0.0
        for c in sorted({0, self.C - 1}):
            I = self.I[c][:, idx].float().cpu().numpy().astype(np.float64)
            ref = o.fit_shared(I, self.pinv64)
            got = self.coef_pk(c)[idx].cpu().numpy()
            worst = max(worst, coef_parity(got, ref))
            rref, _ = o.fit_residual(I, self.A64, ref)
            rg = self.res[c][idx].cpu().numpy()
            worst_r = max(worst_r, float((np.abs(rg - rref) / np.maximum(rref, 1.0)).max()))
        return {"max_rel": worst, "residual_max_rel": worst_r, "tol": 1e-4,
                "ok": bool(worst <= 1e-4 and worst_r <= 1e-4), "checked_px": int(len(idx)),
                "vs": "oracle fit_shared + fit_residual (fp64)"}


class RelightWorkload(Workload):
    """One step = one rti_relight launch evaluating ONE (lu, lv) over this rank's 4K coefficient rows
    (interactive).  Cold (default): launches rotate over `--map-sets` coefficient-map sets and outputs,
    so the bytes touched between two uses of one map exceed the 256 MiB Infinity Cache and every launch
    streams from HBM (MI355X_MICROARCH.md §Infinity Cache); --map-sets 1 measures the L3-resident case."""

    def __init__(self, args, cfg, ctx):
        import torch

        import rti

        self.rti, self.args, self.ctx = rti, args, ctx
        _, H, W, E, C, basis, desc = cfg
        self.W, self.E, self.desc, self.basis = W, E, desc, basis
        self.k = k = rti.basis_terms(basis)
        self.P = P = ctx.h * W
        dev = ctx.dev
        self.sets = max(1, args.map_sets)
        g = torch.Generator(device=dev).manual_seed(1000 + ctx.rank)
        self.coefs = []
        for _ in range(self.sets):
            c = (torch.rand((P, k), generator=g, device=dev) * 100 - 50).contiguous()
            c[:, k - 1] += 130
            self.coefs.append(c)
        rng = np.random.default_rng(4)
        r = np.sqrt(rng.random(E))
        th = 2 * np.pi * rng.random(E)
        self.luv_host = np.stack([r * np.cos(th), r * np.sin(th)], -1)
        self.luv = torch.as_tensor(self.luv_host, device=dev).contiguous()
        self.outs = [torch.empty((P,), dtype=torch.float32, device=dev) for _ in range(self.sets)]
        self.units = P
        self.total_units = ctx.H * W
        self.alg_bytes = 4.0 * P * k + 4.0 * P  # coefficients read + fp32 image written, per eval
        self.metric = f"Mpix*evals/sec {desc}"
        self.unit = "Mpix*evals/s"
        L = rti._lib
        self.L, self.lib, self.bid = L, L.lib(), rti.basis_id(basis)
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def step(self, i):
        L, s = self.L, i % self.sets
        st = self.lib.rti_relight(ctypes.c_void_p(self.coefs[s].data_ptr()), L.RTI_F32, self.bid, self.P,
                                  L.RTI_COEF_PIXEL_MAJOR, ctypes.c_void_p(self.luv.data_ptr() + 16 * (i % self.E)), 1,
                                  ctypes.c_void_p(self.outs[s].data_ptr()), L.RTI_F32, L.RTI_OUT_EVAL_MAJOR,
                                  self.stream)
        if st:
            L.check(st, "rti_relight")

    def config(self):
        return {"evals": self.E, "basis": self.basis, "k": self.k, "coef_layout": "pixel", "out": "f32",
                "map_sets": self.sets, "cache": "cold (working set between reuses > 256 MiB L3)" if self.cold()
                else "L3-resident (one map set re-read every launch)"}

    def cold(self):
        return self.sets * (self.alg_bytes) > 300 * 2 ** 20

    def roofline(self, kernel_ms):
        r = super().roofline(kernel_ms)
        if not self.cold():
            r["bound"] = "l3"  # the maps stay in the 256 MiB Infinity Cache between launches
        return r

    def traffic(self):
        # PMC bytes per launch of the cold (HBM-streamed) case, profiles/traffic.json (tools/pmc_pass.sh)
        if self.ctx.world != 1 or self.ctx.weak or not self.cold():
            return None
        return load_traffic(self.args.config)

    def parity(self):
        import torch

        o = oracle()
        self.step(7)
        torch.cuda.synchronize(self.ctx.dev)
        s = 7 % self.sets
        idx = sample_idx(self.P, 65536, 5)
        lu, lv = self.luv_host[7 % self.E]
        ref = o.relight(self.coefs[s][idx].cpu().numpy(), self.basis, lu, lv)[0]
        got = self.outs[s][idx].cpu().numpy()
        err = float((np.abs(got - ref) / np.maximum(np.abs(ref), 255)).max())
        return {"max_rel": err, "tol": 1e-4, "ok": bool(err <= 1e-4), "checked_px": int(len(idx)),
                "vs": "oracle relight (fp64)"}

    def cpu_fn(self):
        o = oracle()
        rows = max(1, min(self.ctx.h, 216))
        c = self.coefs[0][: rows * self.W].cpu().numpy()
        lu, lv = self.luv_host[0]
        return (lambda: o.relight(c, self.basis, lu, lv), rows * self.W,
                f"oracle relight (fp64 NumPy) on {rows}x{self.W} px x 1 eval")


class FrameWorkload(RelightWorkload):
    """One step = one rti_relight_frame launch: the image relighting_event shows for one cursor position
    (interactive_relighting.py:31-38), from device-resident coefficient maps and HSV ROI."""

    def __init__(self, args, cfg, ctx):
        import torch

        super().__init__(args, cfg, ctx)
        dev = ctx.dev
        g = torch.Generator(device=dev).manual_seed(2000 + ctx.rank)
        self.hsv = torch.randint(0, 256, (self.P, 3), generator=g, device=dev, dtype=torch.uint8)
        self.bgrs = [torch.empty((self.P, 3), dtype=torch.uint8, device=dev) for _ in range(self.sets)]
        self.alg_bytes = 4.0 * self.P * self.k + 3.0 * self.P + 3.0 * self.P  # coefficients + HSV in, BGR out
        self.dtype = "f32 eval -> u8 BGR"

    def step(self, i):
        L, s = self.L, i % self.sets
        lu, lv = self.luv_host[i % self.E]
        st = self.lib.rti_relight_frame(ctypes.c_void_p(self.coefs[s].data_ptr()), L.RTI_F32, self.bid,
                                        L.RTI_COEF_PIXEL_MAJOR, self.P, float(lu), float(lv),
                                        ctypes.c_void_p(self.hsv.data_ptr()), ctypes.c_void_p(self.bgrs[s].data_ptr()),
                                        self.stream)
        if st:
            L.check(st, "rti_relight_frame")

    def config(self):
        c = super().config()
        c.update({"events": self.E, "out": "uint8 BGR [P][3]"})
        c.pop("evals", None)
        return c

    def parity(self):
        import torch

        o = oracle()
        self.step(7)
        torch.cuda.synchronize(self.ctx.dev)
        s = 7 % self.sets
        rows = min(self.ctx.h, 32)
        n = rows * self.W
        lu, lv = self.luv_host[7 % self.E]
        v = o.relight(self.coefs[s][:n].cpu().numpy(), self.basis, lu, lv).reshape(rows, self.W)
        ref = o.relighting_event_image(np.trunc(v).astype(np.int32), self.hsv[:n].cpu().numpy().reshape(rows, self.W, 3))
        got = self.bgrs[s][:n].cpu().numpy().reshape(rows, self.W, 3)
        near = np.abs(v - np.round(v)) < 1e-4  # fp32 evaluation vs fp64 truncation
        bad = (got != ref).any(-1) & ~near
        return {"mismatch_not_near_integer": int(bad.sum()), "checked_px": int(n), "ok": bool(not bad.any()),
                "vs": "oracle relight + clip + HSV2BGR restatement"}

    def cpu_fn(self):
        o = oracle()
        rows = max(1, min(self.ctx.h, 216))
        c = self.coefs[0][: rows * self.W].cpu().numpy()
        hsv = self.hsv[: rows * self.W].cpu().numpy().reshape(rows, self.W, 3)
        lu, lv = self.luv_host[0]

        def one():
            v = o.relight(c, self.basis, lu, lv).reshape(rows, self.W)
            return o.relighting_event_image(np.trunc(v).astype(np.int32), hsv)

        return one, rows * self.W, f"oracle relight + clip + HSV2BGR (NumPy) on {rows}x{self.W} px x 1 event"


class PerPixelWorkload(Workload):
    """One step = one rti_fit_perpixel_cam launch (directions from cameras, fp64 normal equations)."""

    dtype = "f32 in / f64 solve"

    def traffic(self):
        if self.ctx.world != 1 or self.ctx.weak:
            return None
        return load_traffic(self.args.config)

    def __init__(self, args, cfg, ctx):
        import torch

        import rti

        self.rti, self.args, self.ctx = rti, args, ctx
        _, H, W, N, C, basis, desc = cfg
        self.W, self.N, self.desc = W, N, desc
        self.P = P = ctx.h * W
        dev = ctx.dev
        self.cams = synth_cams(N, 6, ctx.H, W)
        lu, lv = synth_dirs(N, seed=2)
        self.I = synth_stack(ctx.H, W, N, 1, "ptm", lu, lv, seed=1000, device=dev, rows=(ctx.r0, ctx.r1))[0]
        self.cams_d = torch.as_tensor(self.cams, device=dev).contiguous()
        self.coef = torch.empty((P, 6), dtype=torch.float32, device=dev)
        self.units = P * N
        self.total_units = ctx.H * W * N
        self.alg_bytes = 4.0 * P * N + 4.0 * P * 6
        self.metric = f"Mpix*lights/sec {desc}"
        self.unit = "Mpix*lights/s"
        L = rti._lib
        fn = L.lib().rti_fit_perpixel_cam
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        cargs = (ctypes.c_void_p(self.cams_d.data_ptr()), N, ctypes.c_void_p(self.I.data_ptr()), L.RTI_F32, ctx.h, W,
                 P, 0.0, float(ctx.r0), -1.0, ctypes.c_void_p(self.coef.data_ptr()), L.RTI_F32,
                 L.RTI_COEF_PIXEL_MAJOR, stream)

        def step(i):
            st = fn(*cargs)
            if st:
                L.check(st, "rti_fit_perpixel_cam")

        self.step = step

    def config(self):
        return {"lights": self.N, "basis": "ptm", "k": 6, "coef_layout": "pixel", "geometry": "per-pixel cameras"}

    def parity(self):
        o = oracle()
        idx = sample_idx(self.P, 2048, 17)
        ys, xs = np.divmod(idx, self.W)
        lu, lv = o.light_dirs_for_pixels(self.cams, xs, ys + self.ctx.r0)
        ref = o.fit_perpixel(lu, lv, self.I[:, idx].cpu().numpy().T)
        err = coef_parity(self.coef[idx].cpu().numpy(), ref)
        return {"max_rel": err, "tol": 1e-4, "ok": bool(err <= 1e-4), "checked_px": int(len(idx)),
                "vs": "oracle fit_perpixel (batched fp64 SVD, reference semantics)"}

    def cpu_fn(self):
        o = oracle()
        npx = min(4096, self.P)
        ys, xs = np.divmod(np.arange(npx), self.W)
        lu, lv = o.light_dirs_for_pixels(self.cams, xs, ys + self.ctx.r0)
        I = self.I[:, :npx].cpu().numpy().T
        return (lambda: o.fit_perpixel(lu, lv, I), npx * self.N,
                f"oracle fit_perpixel (batched fp64 NumPy SVD, reference semantics) on {npx} px x {self.N} lights")


def grid_queries():
    xf = np.around(np.mgrid[-1:1:0.02, -1:1:0.02][1], 2)[0]
    return np.tile(xf, xf.size), np.repeat(xf, xf.size)


class OperatorWorkload(Workload):
    """One step = one rti_apply_operator launch: RBF operator (E = 100x100 grid) over this rank's ROI rows -> int32."""

    def __init__(self, args, cfg, ctx):
        import torch

        import rti

        self.rti, self.args, self.ctx = rti, args, ctx
        _, H, W, N, C, basis, desc = cfg
        self.W, self.N, self.desc = W, N, desc
        self.P = P = ctx.h * W
        dev = ctx.dev
        self.lu, self.lv = synth_dirs(N, seed=2)
        self.I = synth_stack(ctx.H, W, N, 1, "ptm", self.lu, self.lv, seed=1000, device=dev,
                             rows=(ctx.r0, ctx.r1))[0]  # [N, P]
        self.qu, self.qv = grid_queries()
        self.E = E = self.qu.size
        self.op64 = rti.rbf_operator(self.lu, self.lv, self.qu, self.qv)  # [N, E] fp64 (host, one-time)
        self.precision = args.op_precision
        self.op = torch.as_tensor(self.op64.astype(np.float32), device=dev).contiguous()
        if self.precision == "split16":
            self.hi, self.lo, self.Kp, self.inv = rti.api.split_operator_f16(self.op64, dev)
        self.out = torch.empty((E, P), dtype=torch.int32, device=dev)
        self.units = P * E
        self.total_units = ctx.H * W * E
        self.alg_bytes = 4.0 * P * N + 4.0 * P * E  # stack read once + int32 tables written
        self.flops = 2.0 * E * N * P
        self.metric = f"Mpix*evals/sec {desc}"
        self.unit = "Mpix*evals/s"
        self.dtype = ("f32 operator as 2 x f16 (f16 MFMA, f32 accumulate) -> int32" if self.precision == "split16"
                      else "f32 (MFMA) -> int32")
        L = rti._lib
        self.L, self.lib = L, L.lib()
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def step(self, i):
        c, L = ctypes, self.L
        if self.precision == "split16":
            st = self.lib.rti_apply_operator_f16(c.c_void_p(self.hi.data_ptr()), c.c_void_p(self.lo.data_ptr()),
                                                 self.Kp, self.inv, self.E, self.N, c.c_void_p(self.I.data_ptr()),
                                                 L.RTI_F32, self.P, 1, self.P, self.N * self.P,
                                                 c.c_void_p(self.out.data_ptr()), L.RTI_I32, self.P, self.E * self.P,
                                                 self.stream)
            if st:
                L.check(st, "rti_apply_operator_f16")
            return
        st = self.lib.rti_apply_operator(c.c_void_p(self.op.data_ptr()), self.E, self.N, self.E,
                                         c.c_void_p(self.I.data_ptr()), L.RTI_F32, self.P, 1, self.P, self.N * self.P,
                                         c.c_void_p(self.out.data_ptr()), L.RTI_I32, self.P, self.E * self.P, self.stream)
        if st:
            L.check(st, "rti_apply_operator")

    def config(self):
        return {"lights": self.N, "evals": self.E, "basis": "rbf-linear", "out": "int32 tables [E][P]",
                "operator_precision": self.precision}

    def traffic(self):
        if self.ctx.world != 1 or self.ctx.weak:
            return None
        return load_traffic(f"{self.args.config}-{self.precision}")

    def roofline(self, kernel_ms):
        ach = self.flops / (kernel_ms * 1e-3) / 1e12
        if self.precision == "split16":
            # two f16 MFMA products per multiply-add put the compute at 2 x 3.2e11 x 1.12 flop per launch
            # (~0.3 ms at the dense f16 peak), so the E x P int32 table writes (6.4 GB) bound it: HBM roofline
            r = super().roofline(kernel_ms)
            r.update({"alg_flops_per_launch": self.flops,
                      "mfma_f16_TFLOPs_issued": round(2 * self.flops * (self.Kp / self.N) / (kernel_ms * 1e-3) / 1e12, 1),
                      "mfma_f16_peak": 2516.6})
            return r
        return {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / MFMA_F32_PEAK_TFLOPS, 4), "traffic": None, "kernel_ms": round(kernel_ms, 4),
                "alg_flops_per_launch": self.flops, "alg_bytes_per_launch": self.alg_bytes,
                "hbm_GBps": round(self.alg_bytes / (kernel_ms * 1e-3) / 1e9, 1)}

    def parity(self):
        idx = sample_idx(self.P, 512, 19)
        ref = self.op64.T @ self.I[:, idx].cpu().numpy().astype(np.float64)  # [E, n]
        got = self.out[:, idx].cpu().numpy()
        r = int_table_parity(got, ref)
        r["vs"] = "fp64 operator product (oracle rbf_operator-equivalent) truncated to int32"
        return r

    def cpu_fn(self):
        npx = min(256, self.P)
        I = self.I[:, :npx].cpu().numpy().astype(np.float64)
        op = self.op64
        return (lambda: (op.T @ I).astype(np.int32), npx * self.E,
                f"NumPy fp64 operator product (the SciPy-Rbf-equivalent grid) on {npx} px x {self.E} evals")


class RbfPerPixelWorkload(Workload):
    """One step = one rti_rbf_perpixel launch over this rank's ROI rows: per-pixel fp64 solve + 10^4 evaluations."""

    dtype = "f64 -> int32"

    def __init__(self, args, cfg, ctx):
        import torch

        import rti

        self.rti, self.args, self.ctx = rti, args, ctx
        _, H, W, N, C, basis, desc = cfg
        self.W, self.N, self.desc = W, N, desc
        self.P = P = ctx.h * W
        dev = ctx.dev
        cams = synth_cams(N, 6, ctx.H, W)
        ys, xs = np.divmod(np.arange(P), W)
        ys = ys + ctx.r0
        dx = cams[None, :, 0] - xs[:, None]
        dy = cams[None, :, 1] - ys[:, None]
        nrm = np.sqrt(dx * dx + dy * dy + cams[None, :, 2] ** 2)
        self.lu_h = (dx / nrm).astype(np.float32)
        self.lv_h = (dy / nrm).astype(np.float32)
        self.lu = torch.as_tensor(self.lu_h, device=dev)
        self.lv = torch.as_tensor(self.lv_h, device=dev)
        rng = np.random.default_rng(7 + ctx.rank)
        self.I_h = rng.integers(0, 256, (P, N)).astype(np.int32)
        self.I = torch.as_tensor(self.I_h, device=dev)
        self.qu, self.qv = grid_queries()
        self.E = E = self.qu.size
        self.luv = torch.as_tensor(np.stack([self.qu, self.qv], -1), device=dev).contiguous()
        self.out = torch.empty((E, P), dtype=torch.int32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.units = P * E
        self.total_units = ctx.H * W * E
        self.alg_bytes = 12.0 * P * N + 4.0 * P * E
        self.flops = P * (2.0 / 3.0 * N ** 3 + 5.0 * N * N + 8.0 * N * E)  # LU + A build + evaluation (fp64)
        self.metric = f"Mpix*evals/sec {desc}"
        self.unit = "Mpix*evals/s"
        L = rti._lib
        self.L, self.lib = L, L.lib()
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def step(self, i, fallback=None):
        c, L = ctypes, self.L
        st = self.lib.rti_rbf_perpixel_ex(c.c_void_p(self.lu.data_ptr()), c.c_void_p(self.lv.data_ptr()),
                                          c.c_void_p(self.I.data_ptr()), L.RTI_I32, self.N, self.P,
                                          c.c_void_p(self.luv.data_ptr()), self.E, c.c_void_p(self.out.data_ptr()),
                                          L.RTI_I32, L.RTI_OUT_EVAL_MAJOR, c.c_void_p(self.status.data_ptr()),
                                          c.c_void_p(fallback.data_ptr() if fallback is not None else None),
                                          self.stream)
        if st:
            L.check(st, "rti_rbf_perpixel_ex")

    def fallback_px(self):
        """Pixels one step hands to the fp64 partial-pivoting fallback (81 <= N <= 256; 0 otherwise)."""
        import torch

        cnt = torch.zeros(1, dtype=torch.int32, device=self.I.device)
        self.step(0, cnt)
        torch.cuda.synchronize(self.I.device)
        return int(cnt.item())

    def config(self):
        return {"lights": self.N, "evals": self.E, "basis": "rbf-linear per-pixel", "out": "int32 tables [E][P]",
                "fallback_px": self.fallback_px()}

    def roofline(self, kernel_ms):
        ach = self.flops / (kernel_ms * 1e-3) / 1e12
        return {"bound": "fp64-valu", "achieved": round(ach, 2), "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP64_VALU_PEAK_TFLOPS, 4), "traffic": None, "kernel_ms": round(kernel_ms, 4),
                "alg_flops_per_launch": self.flops, "alg_bytes_per_launch": self.alg_bytes}

    def parity(self):
        o = oracle()
        idx = sample_idx(self.P, 8, 23)
        ref = np.stack([o.rbf_linear(self.lu_h[p], self.lv_h[p], self.I_h[p], self.qu, self.qv) for p in idx], -1)
        got = self.out[:, idx].cpu().numpy()
        r = int_table_parity(got, ref)
        r["vs"] = "oracle rbf_linear (SciPy-equivalent fp64 solve + cdist eval)"
        return r

    def cpu_fn(self):
        o = oracle()
        npx = 16

        def run():
            for p in range(npx):
                o.rbf_linear(self.lu_h[p], self.lv_h[p], self.I_h[p], self.qu, self.qv)

        return run, npx * self.E, f"oracle rbf_linear (SciPy-equivalent fp64 solve + cdist eval) on {npx} px x {self.E} evals"


WORKLOADS = {"fit": FitWorkload, "fit_residual": FitResidualWorkload, "relight": RelightWorkload,
             "perpixel": PerPixelWorkload, "frame": FrameWorkload, "operator": OperatorWorkload,
             "rbf_perpixel": RbfPerPixelWorkload}


# ---- CPU baseline -----------------------------------------------------------------------------

def cgroup_cpus():
    """CPUs granted by the cgroup quota (cpu.max), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def time_cpu(fn, units, budget_s):
    """1 warm-up, then repeats until >= 5 runs and >= budget_s; rate from the median run."""
    fn()
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < 5 or time.perf_counter() < t_end:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    return units / float(np.median(times)) / 1e6, len(times)


def cpu_baseline(wl, budget_s):
    from threadpoolctl import threadpool_limits

    fn, units, desc = wl.cpu_fn()
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    threads = min(aff, quota) if quota else aff
    with threadpool_limits(threads):
        rate_n, reps_n = time_cpu(fn, units, budget_s / 2)
    with threadpool_limits(1):
        rate_1, reps_1 = time_cpu(fn, units, budget_s / 2)
    out = {"value": round(rate_n, 3), "unit": wl.unit, "cores": threads, "kind": "port",
           "value_1thread": round(rate_1, 3),
           "sample": f"{desc}; median of {reps_n} runs at {threads} BLAS threads (sched_getaffinity {aff}"
                     f"{f', cgroup quota {quota}' if quota else ''}) and of {reps_1} runs at 1 thread, after 1 "
                     f"warm-up each; {cpu_model()}"}
    ref = getattr(wl, "cpu_ref_fn", None)
    if ref is not None:  # the reference's own per-pixel SVD semantics, beside the port
        fn, units, desc = ref()
        with threadpool_limits(threads):
            rr_n, rn = time_cpu(fn, units, budget_s / 4)
        with threadpool_limits(1):
            rr_1, r1 = time_cpu(fn, units, budget_s / 4)
        out["reference_semantics"] = {
            "value": round(rr_n, 3), "unit": wl.unit, "cores": threads, "value_1thread": round(rr_1, 3),
            "kind": "reference-semantics port",
            "sample": f"{desc}; median of {rn} runs at {threads} BLAS threads and of {r1} runs at 1 thread, after 1 "
                      f"warm-up each; {cpu_model()}"}
        out["note"] = ("value = the build's vectorised port (one shared fp64 pinv, fp32 matmul); "
                       "reference_semantics = the reference's per-pixel SVD least squares (analysis.py:280-298)")
    return out


# ---- multi-GPU legs ---------------------------------------------------------------------------

def cyclic_stack(wl, ctx, chunks):
    """This rank's rows under the block-cyclic partition (rti.parallel.cyclic_rows), generated on the
    device block by block exactly as the block rows are (synth_stack is a function of the global rows),
    every channel, in the workload's intensity dtype and stack layout: light-major [C, N, h, W] (C = 1:
    [N, h, W]) or the reference's pixel-major [C, h, W, N] ([h, W, N])."""
    import torch

    from rti.parallel import cyclic_rows

    blocks = cyclic_rows(ctx.H, ctx.world, ctx.rank, chunks)
    parts = [synth_stack(ctx.H, wl.W, wl.N, wl.C, wl.basis, wl.lu, wl.lv, seed=1000, device=ctx.dev, rows=b)
             for b in blocks]
    I = torch.cat(parts, dim=2).reshape(wl.C, wl.N, -1, wl.W)
    del parts
    if I.dtype != wl.I.dtype:
        I = I.to(wl.I.dtype)
    if wl.stack == "pixel":
        I = I.permute(0, 2, 3, 1).contiguous()
    return I if wl.C > 1 else I[0]


def e2e_parity(wl, ctx, full, chunks, per_block=256):
    """Rank 0: sampled pixels of EVERY row block of the gathered map (all ranks' blocks, block-cyclic
    order; channels 0 and C - 1) against the oracle on that block's regenerated intensities — checks the
    fit and that every block landed in its place."""
    from rti.parallel import cyclic_rows

    o = oracle()
    worst, checked = 0.0, 0
    fullc = full if wl.C > 1 else full.unsqueeze(0)
    for r in range(ctx.world):
        for bi, (r0, r1) in enumerate(cyclic_rows(ctx.H, ctx.world, r, chunks)):
            I = synth_stack(ctx.H, wl.W, wl.N, wl.C, wl.basis, wl.lu, wl.lv, seed=1000, device=ctx.dev, rows=(r0, r1))
            if wl.in_bytes == 1:
                I = I.to(wl.I.dtype)
            idx = sample_idx((r1 - r0) * wl.W, per_block, 17 + 31 * r + bi)
            for c in sorted({0, wl.C - 1}):
                ref = o.fit_shared(I[c][:, idx].float().cpu().numpy(), wl.pinv64)
                got = fullc[c][r0:r1].reshape(-1, wl.k)[idx].cpu().numpy()
                worst = max(worst, coef_parity(got, ref))
                checked += len(idx)
    return {"max_rel": worst, "tol": 1e-4, "ok": bool(worst <= 1e-4), "checked_px": checked,
            "blocks": ctx.world * chunks, "vs": "oracle fit_shared on each block's regenerated rows"}


def allgather_legs(wl, ctx, reps=5):
    """RCCL all-gather of this rank's coefficient rows into the whole [H, W, k] map, and the row-chunked
    fit with each chunk's all-gather overlapped with the next chunk's fit (block-cyclic rows, so every
    chunk lands in place; this rank's cyclic rows are generated for it).  Returns (allgather_ms,
    overlapped_ms, chunks, e2e parity of the overlapped map; rank 0 checks, others None)."""
    import torch
    import torch.distributed as dist

    from rti.parallel import RowTiledFitter, gather_rows

    dev = ctx.dev
    locals_ = [(wl.coef[c].reshape(ctx.h, wl.W, wl.k) if wl.args.layout == "pixel" else
                wl.coef[c].T.reshape(ctx.h, wl.W, wl.k).contiguous()) for c in range(wl.C)]

    def gather_all():  # every channel's rows (one collective per channel)
        for loc in locals_:
            gather_rows(loc, ctx.H)
    for _ in range(2):
        gather_all()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        gather_all()
    torch.cuda.synchronize(dev)
    gather_ms = (time.perf_counter() - t0) / reps * 1e3
    # cyclic blocks of H/(G*chunks) rows (4K on 8 GPUs: 2160/8 = 270 rows per rank -> 3 chunks of 90)
    if ctx.H % ctx.world:  # the block-cyclic leg needs equal row blocks on every rank
        return gather_ms, None, 0, {"skipped": f"H={ctx.H} is not a multiple of {ctx.world} ranks", "ok": True}
    chunks = next((c for c in (4, 3, 2, 1) if ctx.H % (ctx.world * c) == 0), 1)
    I_cyc = cyclic_stack(wl, ctx, chunks)
    # the same kernel family as the 1-GPU line: every channel, the stack's layout (rti_fit_shared_pm for the
    # reference's pixel-major stacks), 8-bit stacks on the h16 matrix-core fit
    fitter = RowTiledFitter(I_cyc, wl.lu, wl.lv, ctx.H, basis=wl.basis, chunks=chunks, partition="cyclic",
                            stack=wl.stack, kernel=wl.args.kernel)
    for _ in range(2):
        fitter()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        full = fitter()
    torch.cuda.synchronize(dev)
    e2e_ms = (time.perf_counter() - t0) / reps * 1e3
    par = None
    if not wl.args.no_parity and ctx.rank == 0:
        par = e2e_parity(wl, ctx, full, chunks)
    del I_cyc, fitter
    return gather_ms, e2e_ms, chunks, par


def device_info(dev):
    """The box this line was measured on (box-to-box spread is ~±6 %)."""
    import torch

    p = torch.cuda.get_device_properties(dev)
    return {"name": p.name, "arch": getattr(p, "gcnArchName", ""), "cus": p.multi_processor_count,
            "hbm_GiB": round(p.total_memory / 2 ** 30, 1)}


def reduce_max(vals, ctx, backend):
    import torch
    import torch.distributed as dist

    t = torch.tensor(vals, dtype=torch.float64, device=ctx.dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]


def gather_vals(v, ctx, backend):
    import torch
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.float64, device=ctx.dev if backend == "nccl" else "cpu")
    out = [torch.empty_like(t) for _ in range(ctx.world)]
    dist.all_gather(out, t)
    return [float(x[0]) for x in out]


# ---- main -------------------------------------------------------------------------------------

def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 20 (fit) / 1000 (relight) / 10 (per-pixel)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--weak", action="store_true", help="every rank fits a whole H-row image (weak scaling)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "valu", "mfma", "tile", "q8", "h16"])
    ap.add_argument("--layout", default="pixel", choices=["pixel", "planar"])
    ap.add_argument("--stack", default="light", choices=["light", "pixel"],
                    help="fit configs: intensity stack layout; pixel = the reference's (R, R, N) (rti_fit_shared_pm)")
    ap.add_argument("--nontemporal", action="store_true")
    ap.add_argument("--in-dtype", default="f32", choices=["f32", "u8", "i32"],
                    help="intensity stack type for fit configs (BASELINE's metric is fp32)")
    ap.add_argument("--op-precision", default="split16", choices=["split16", "fp32"],
                    help="c7: operator as two fp16 halves on f16 MFMA (default) or fp32 on f32 MFMA")
    ap.add_argument("--map-sets", type=int, default=3,
                    help="c5/c9: coefficient-map sets rotated over launches (3 = HBM-cold, 1 = L3-resident)")
    ap.add_argument("--no-allgather", action="store_true", help="N>1: skip the RCCL all-gather legs")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-parity", action="store_true", help="skip the in-run parity check")
    ap.add_argument("--cpu-budget", type=float, default=16.0, help="seconds of CPU baseline (half per thread count)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for real runs; gloo lets ranks share one GPU in rehearsals")
    ap.add_argument("--shape", default=None,
                    help="HxW override of the config's image (rehearsals and tests only; the line's config says it)")
    ap.add_argument("--plan", action="store_true",
                    help="print the rank/row plan only (no device work; CPU tests of the launcher)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    maybe_spawn(args)
    cfg = CONFIGS[args.config]
    if args.shape:
        h, w = (int(x) for x in args.shape.lower().split("x"))
        cfg = (cfg[0], h, w) + cfg[3:6] + (cfg[6] + f" [shape override {h}x{w}]",)
    kind = cfg[0]
    if args.stack == "pixel" and kind != "fit":
        raise SystemExit("--stack pixel applies to the fit configs (c2, c3, c4)")
    if args.kernel in ("q8", "h16") and (kind not in ("fit",) or args.in_dtype != "u8"):
        raise SystemExit(f"--kernel {args.kernel} is the 8-bit fit: it needs a fit config and --in-dtype u8")
    auto_steps = args.steps is None
    if auto_steps:
        args.steps = DEFAULT_STEPS[kind]

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = "gloo" if args.plan else args.dist_backend
    if args.plan:
        dev = torch.device("cpu")
    else:
        ndev = max(1, torch.cuda.device_count())
        dev = torch.device("cuda", local % ndev)
        torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    ctx = Ctx(args, cfg[1], rank, world, dev)
    if args.plan:
        rows = [[int(a), int(b)] for a, b in zip(gather_vals(ctx.r0, ctx, "gloo"), gather_vals(ctx.r1, ctx, "gloo"))] \
            if world > 1 else [[ctx.r0, ctx.r1]]
        if rank == 0:
            print(json.dumps({"metric": None, "value": None, "n_gpus": world, "plan_only": True,
                              "scaling": "weak" if args.weak else "strong",
                              "config": {"workload": cfg[6], "H": ctx.H, "W": cfg[2], "H_per_rank": ctx.h,
                                         "rows_per_rank": rows}}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    import rti

    rti.load()
    wl = WORKLOADS[kind](args, cfg, ctx)
    torch.cuda.synchronize(dev)

    tw = time.perf_counter()
    for i in range(args.warmup):
        wl.step(i)
    torch.cuda.synchronize(dev)
    if auto_steps and args.warmup > 1:
        # no --steps: enough steps for a timed region of >= 50 ms, so short kernels (u8, c2: 0.03-0.2 ms) are not
        # dominated by the region's first launch and last sync (same count on every rank: the max is taken)
        est = (time.perf_counter() - tw) / args.warmup
        want = int(np.ceil(0.05 / max(est, 1e-6)))
        if world > 1:
            want = int(reduce_max([float(want)], ctx, backend)[0])
        args.steps = max(args.steps, min(want, 5000))

    stream = torch.cuda.current_stream(dev)
    # timed region: exactly K steps between barrier + synchronize, nothing else enqueued
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        wl.step(i)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0  # this rank's K steps; the max over ranks is taken below
    if world > 1:
        dist.barrier()

    # per-launch spread (kernel_ms_stats): HIP events around each launch on the launch stream,
    # 10 warm-ups then 50 pairs, in a separate pass so the events add no gaps above
    for i in range(10):
        wl.step(i)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for i, (a, b) in enumerate(ev):
        a.record(stream)
        wl.step(i)
        b.record(stream)
    torch.cuda.synchronize(dev)
    kms = np.array([a.elapsed_time(b) for a, b in ev])
    # the roofline's launch duration (median of 50 after 10 warm-ups): 50 event-pair
    # windows of m back-to-back launches each, m sized so a window holds ≥ 1 ms of work.  An event
    # pair adds ≈4 µs per window (10 % of a 40 µs relight when m = 1); rocprofv3's kernel-trace
    # average has no such overhead, and the windowed median agrees with it
    m = max(1, int(np.ceil(1.0 / max(float(np.median(kms)), 1e-3))))
    wms = kms  # a launch ≥ 1 ms: the per-launch pairs already are the windows
    if m > 1:
        win = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
        for a, b in win:
            a.record(stream)
            for i in range(m):
                wl.step(i)
            b.record(stream)
        torch.cuda.synchronize(dev)
        wms = np.array([a.elapsed_time(b) / m for a, b in win])
    kernel_ms = float(np.median(wms))
    kernel_ms_rank = [kernel_ms]
    if world > 1:
        kernel_ms_rank = gather_vals(kernel_ms, ctx, backend)
        elapsed, kernel_ms = reduce_max([elapsed, kernel_ms], ctx, backend)

    parity = None
    if not args.no_parity:
        parity = wl.parity()
        if world > 1:  # every rank checked its own rows; report the worst
            worst = reduce_max([parity.get("max_rel", 0.0), 0.0 if parity["ok"] else 1.0], ctx, backend)
            if "max_rel" in parity:
                parity["max_rel"] = worst[0]
            parity["ok"] = worst[1] == 0.0
            parity["ranks"] = world

    gather_ms = e2e_ms = e2e_par = None
    if world > 1 and kind == "fit" and not args.no_allgather:
        gather_ms, e2e_ms, n_chunks, e2e_par = allgather_legs(wl, ctx)
        gather_ms, e2e_ms = reduce_max([gather_ms, e2e_ms if e2e_ms is not None else 0.0], ctx, backend)
        e2e_ms = e2e_ms or None

    value = wl.total_units * args.steps / elapsed / 1e6
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(wl, args.cpu_budget)
    if rank == 0:
        conf = {"workload": wl.desc, "H": ctx.H, "W": wl.W, "H_per_rank": ctx.h}
        conf.update(wl.config())
        conf["parallelism"] = (f"row-tiled x{world}: rank r fits rows [r*H/G, (r+1)*H/G) of one {ctx.H}-row image"
                               if not args.weak else f"row-tiled x{world}: one {ctx.h}-row image per GPU (weak)")
        line = {
            "metric": wl.metric,
            "value": round(value, 1),
            "unit": wl.unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": wl.dtype,
            "data": "synthetic (seeded smooth PTM/HSH coefficient fields + N(0,2) noise, rounded to 0..255, fp32)",
            "config": conf,
            # the same work over the event-timed kernel time (median of 50 windows of >= 1 ms): a timed region of
            # K short steps carries the launch/sync overhead of its first and last step, this figure does not
            "value_kernel": round(wl.total_units / (kernel_ms * 1e-3) / 1e6, 1),
            "timed_region_ms": round(elapsed * 1e3, 3),
            "roofline": wl.roofline(kernel_ms),
            "kernel_ms_stats": {"median": round(kernel_ms, 5), "min": round(float(wms.min()), 5),
                                "mean": round(float(wms.mean()), 5), "n": 50, "launches_per_window": m,
                                "warmup": 10, "per_launch_median": round(float(np.median(kms)), 5),
                                "per_launch_min": round(float(kms.min()), 5),
                                "per_launch_mean": round(float(kms.mean()), 5), "per_launch_n": int(kms.size),
                                "per_rank_median": [round(x, 5) for x in kernel_ms_rank]},
            "parity": parity,
            "cpu_baseline": cpu,
            "device": device_info(dev),
        }
        if gather_ms is not None:
            line["allgather_ms"] = round(gather_ms, 3)
            if e2e_ms is not None:
                line["fit_allgather_overlapped_ms"] = round(e2e_ms, 3)  # row chunks, gather(c) || fit(c+1)
                line["overlap_chunks"] = int(n_chunks)
                line["end_to_end_Mpix_lights_per_s"] = round(wl.total_units / (e2e_ms * 1e-3) / 1e6, 1)
            line["e2e_parity"] = e2e_par
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
