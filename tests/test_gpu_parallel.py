"""Two ranks sharing cuda:0 (gloo coordination) run the row-tiled GPU fit and the
coefficient-map all-gather; the assembled map must equal the single-process fit
row for row.  On an 8-GPU node the same code runs with backend "nccl" (RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import rti
    import rti_oracle as o
    from rti.parallel import fit_rowtiled, fit_rowtiled_overlapped, row_range

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        H, W, N = 37, 64, 30
        lu, lv = o.synth_dirs(N, 3)
        I = o.synth_intensities(H, W, lu, lv, seed=8)
        r0, r1 = row_range(H, world, rank)
        dev = torch.device("cuda", 0)
        local = torch.as_tensor(np.ascontiguousarray(I[:, r0:r1]), device=dev)
        full = fit_rowtiled(local, lu, lv, H).cpu().numpy()
        whole = rti.fit(torch.as_tensor(I, device=dev), lu, lv).cpu().numpy()
        ref = o.fit_shared(I, o.pinv_shared("ptm", lu, lv)).reshape(H, W, 6)
        err = float((np.abs(full - ref) / np.abs(ref).max(-1, keepdims=True)).max())
        over = fit_rowtiled_overlapped(local, lu, lv, H, chunks=3).cpu().numpy()  # chunked fit + all-gather
        same = bool(np.array_equal(full, whole)) and bool(np.array_equal(over, whole))
        q.put((rank, full.shape, same, err))
    finally:
        dist.destroy_process_group()


def test_rowtiled_fit_two_ranks_one_gpu(cuda):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, shape, same, err in results:
        assert shape == (37, 64, 6) and same and err < 1e-4, (rank, shape, same, err)


@pytest.mark.parametrize("gpus,shape,extra", [(2, "96x128", []), (3, "90x64", ["--in-dtype", "u8"]),
                                              (2, "64x96", ["--weak"]), (2, "96x128", ["--stack", "pixel"]),
                                              (3, "48x64", ["--config", "c4"])])
def test_bench_multi_rank_end_to_end_parity(cuda, gpus, shape, extra):
    """bench.py --gpus N (ranks sharing cuda:0 over gloo): the strong-scaling line, the all-gather legs and
    the overlapped row-chunked fit whose gathered map (block-cyclic rows generated per rank) rank 0 checks
    block by block against the oracle (e2e_parity) — on the same kernel family as the 1-GPU line: 8-bit
    stacks on the h16 fit, the reference's pixel-major stack, and all three HSH-16 channels of c4."""
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dist-backend", "gloo",
                        "--config", "c2", "--shape", shape, "--steps", "2", "--warmup", "1", "--no-cpu"] + extra,
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == gpus and line["parity"]["ok"], line["parity"]
    e2e = line["e2e_parity"]
    assert e2e["ok"] and e2e["blocks"] == gpus * line["overlap_chunks"] and e2e["checked_px"] > 0, e2e


def _modes_worker(rank, world, port, partition, q):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "smartphone-based-rti_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import rti
    import rti_oracle as o
    from rti.parallel import RowTiledFitter, cyclic_rows, relight_rowtiled, row_range

    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        dev = torch.device("cuda", 0)
        H, W, chunks = 24, 64, (3 if world == 2 else 2)
        rows = cyclic_rows(H, world, rank, chunks) if partition == "cyclic" else [row_range(H, world, rank)]

        def mine(x, dim):  # this rank's rows of a whole-image tensor, along `dim`
            return torch.cat([x.narrow(dim, a, b - a) for a, b in rows], dim=dim).contiguous()

        rng = np.random.default_rng(5)
        # (1) RGB HSH-16, light-major fp32 [C, N, H, W]
        N = 40
        lu, lv = o.synth_dirs(N, 2)
        I = torch.as_tensor(rng.integers(0, 256, (3, N, H, W)).astype(np.float32), device=dev)
        whole = rti.fit(I, lu, lv, basis="hsh")  # [3, H, W, 16]
        got = RowTiledFitter(mine(I, 2), lu, lv, H, basis="hsh", chunks=chunks, partition=partition)()
        out["rgb_hsh16"] = bool(torch.equal(got, whole))
        # (2) pixel-major stack [C, H, W, N] (the reference's layout), PTM-6
        Ipm = I.permute(0, 2, 3, 1).contiguous()
        whole = rti.fit(Ipm, lu, lv, stack="pixel")
        got = RowTiledFitter(mine(Ipm, 1), lu, lv, H, stack="pixel", chunks=chunks, partition=partition)()
        out["pixel_major"] = bool(torch.equal(got, whole))
        # (3) 8-bit light-major (the V channel): the h16 fit per chunk
        I8 = I[0].to(torch.uint8)
        whole = rti.fit(I8, lu, lv)
        fitter = RowTiledFitter(mine(I8, 1), lu, lv, H, chunks=chunks, partition=partition)
        got = fitter()
        s = whole.abs().amax(-1, keepdim=True).clamp_min(1.0)
        out["u8_h16"] = fitter.u8 == "h16" and float(((got - whole) / s).abs().max()) < 1e-6
        # (3b) the int8 fixed-point fit asked for by name (r06: RowTiledFitter maps kernel="q8" like rti.fit)
        whole = rti.fit(I8, lu, lv, kernel="q8")
        fitter = RowTiledFitter(mine(I8, 1), lu, lv, H, chunks=chunks, partition=partition, kernel="q8")
        out["u8_q8"] = fitter.u8 == "q8" and bool(torch.equal(fitter(), whole))
        # (3c) an integer kernel word reaches rti_fit_shared_pm unmasked (NT_STORE is a documented pm bit)
        kw = rti._lib.RTI_KERNEL_NT_STORE
        whole = rti.fit(Ipm, lu, lv, stack="pixel", kernel=kw)
        got = RowTiledFitter(mine(Ipm, 1), lu, lv, H, stack="pixel", chunks=chunks, partition=partition, kernel=kw)()
        out["pixel_major_kernel_word"] = bool(torch.equal(got, whole))
        # (4) per-pixel camera mode: every chunk's light vectors from its GLOBAL rows (analysis.py:228)
        cams = np.stack([W / 2 + 300 * np.cos(np.linspace(0, 6, N)), H / 2 + 300 * np.sin(np.linspace(0, 6, N)),
                         np.full(N, 400.0)], -1)
        for cdt in (torch.float32, torch.float64):
            whole = rti.fit(I[0], mode="perpixel", cams=cams, origin=(3.0, 5.0), coef_dtype=cdt)
            got = RowTiledFitter(mine(I[0], 1), H=H, mode="perpixel", cams=cams, origin=(3.0, 5.0), chunks=chunks,
                                 partition=partition, coef_dtype=cdt)()
            out[f"perpixel_{cdt}"] = bool(torch.equal(got, whole))
        # (5) relight row shards (block partition), gathered into whole images
        coef = rti.fit(I[0], lu, lv)
        r0, r1 = row_range(H, world, rank)
        whole = rti.relight(coef, [0.1, -0.3], [0.2, 0.5])
        loc = relight_rowtiled(coef[r0:r1].contiguous(), [0.1, -0.3], [0.2, 0.5], H)
        full = relight_rowtiled(coef[r0:r1].contiguous(), [0.1, -0.3], [0.2, 0.5], H, gather=True)
        out["relight"] = bool(torch.equal(loc, whole[:, r0:r1])) and bool(torch.equal(full.to(dev), whole))
        q.put((rank, out))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,partition", [(2, "block"), (3, "block"), (2, "cyclic"), (3, "cyclic")])
def test_rowtiled_modes_match_single_process(cuda, world, partition):
    """"Per-pixel mode shards the same way", "Relight (C5): also row-shardable" — and the
    fit's other stack forms.  Ranks sharing cuda:0 (gloo) fit their rows of RGB HSH-16, pixel-major, 8-bit
    (h16) and per-pixel camera stacks with RowTiledFitter, and relight their rows; every gathered map must
    equal the single-process result (bit for bit; the h16 map within 1e-6 of max|c|)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_modes_worker, args=(r, world, port, partition, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in results:
        assert "error" not in out and all(out.values()), (rank, out)
