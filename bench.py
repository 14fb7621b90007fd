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
    # name: (H, W, lights, channels, basis, description)
    "c2": (1080, 1920, 50, 1, "ptm", "ptm6-fit 1920x1080 N=50 fp32 (BASELINE configs[1])"),
    "c3": (2160, 3840, 100, 1, "ptm", "ptm6-fit 3840x2160 N=100 fp32 (BASELINE configs[2], metric config)"),
    "c4": (2160, 3840, 200, 3, "hsh", "hsh16-fit 3840x2160 RGB N=200 fp32 (BASELINE configs[3])"),
}


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


def cpu_baseline(I_dev, pinv64, N, W, budget_s=10.0):
    """Oracle restatement: fp64 pinv (already built) + fp32 matmul on (N, P) light-major rows."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rti_oracle as o
    try:
        from threadpoolctl import threadpool_info
        threads = max([t.get("num_threads", 1) for t in threadpool_info() if t.get("user_api") == "blas"] or [1])
    except Exception:  # pragma: no cover
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    rows = 216  # a tenth of a 4K frame, all N lights
    sample = I_dev[0, :, : rows * W].cpu().numpy()  # [N, rows*W]
    units = N * rows * W
    o.fit_shared_f32(sample, pinv64)  # warm-up
    t0 = time.perf_counter()
    reps = 0
    while True:
        o.fit_shared_f32(sample, pinv64)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    cpu_name = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": units * reps / el / 1e6, "unit": "Mpix*lights/s", "cores": int(threads), "kind": "port",
            "sample": f"oracle fit_shared_f32 (fp64 pinv + fp32 numpy matmul) on {rows}x{W} px x {N} lights, "
                      f"{reps} reps in {el:.1f}s; {cpu_name}"}


def load_traffic(workload_key):
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            entry = json.load(f).get(workload_key) or {}
        return entry.get("traffic_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--kernel", default="auto", choices=["auto", "valu", "mfma"])
    ap.add_argument("--layout", default="pixel", choices=["pixel", "planar"])
    ap.add_argument("--nontemporal", action="store_true")
    ap.add_argument("--allgather", action="store_true", help="also time the RCCL all-gather of the maps")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    import rti

    rti.load()
    H, W, N, C, basis, desc = CONFIGS[args.config]
    k = rti.basis_terms(basis)
    P = H * W
    lu, lv = synth_dirs(N, seed=2)
    I = synth_stack(H, W, N, C, basis, lu, lv, seed=1000 + rank, device=dev)  # this rank's stripe
    pinv64 = rti.pinv(lu, lv, basis)
    pinv_dev = torch.as_tensor(pinv64.astype(np.float32), device=dev)
    shape = (C, P, k) if args.layout == "pixel" else (C, k, P)
    coef = torch.empty(shape, dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)

    def step():
        rti.fit_shared_into(pinv_dev, I, coef, k=k, layout=args.layout, kernel=args.kernel,
                            nontemporal=args.nontemporal)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])

    gather_ms = None
    if args.allgather and world > 1:
        from rti.parallel import gather_rows

        local_map = coef[0].reshape(H, W, k) if args.layout == "pixel" else coef[0].reshape(k, H, W)
        for _ in range(2):
            gather_rows(local_map, H * world)
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(5):
            gather_rows(local_map, H * world)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) / 5 * 1e3

    units_per_rank = P * N * C  # pixel·lights(·channels) per step
    value = world * units_per_rank * args.steps / elapsed / 1e6
    alg_bytes = 4.0 * P * N * C + 4.0 * P * k * C  # fp32 intensities read + fp32 coefficients written
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    workload_key = f"{args.config}-{args.kernel}-{args.layout}"
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(I, pinv64, N, W, budget_s=args.cpu_budget)
    if rank == 0:
        line = {
            "metric": "Mpix*lights/sec PTM fit (4K, 100 lights)" if args.config == "c3" else f"Mpix*lights/sec {desc}",
            "value": round(value, 1),
            "unit": "Mpix*lights/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded smooth PTM/HSH coefficient fields + N(0,2) noise, rounded to 0..255, fp32)",
            "config": {"workload": desc, "H_per_rank": H, "W": W, "lights": N, "channels": C, "basis": basis,
                       "k": k, "coef_layout": args.layout, "kernel": args.kernel,
                       "parallelism": f"row-stripes x{world} (one {H}-row stripe per GPU)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(workload_key),
                         "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        if gather_ms is not None:
            line["allgather_ms"] = round(gather_ms, 3)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
