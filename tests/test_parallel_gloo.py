"""Row-block sharding + coefficient-map all-gather (rti.parallel) with world_size 2
over gloo on the CPU.  The GPU path uses the same code with backend "nccl" (RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rti.parallel import cyclic_rows, gather_rows, gather_rows_pipelined, row_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("H,world", [(2160, 8), (7, 3), (5, 8), (1, 2), (270, 4)])
def test_row_range_partitions_rows(H, world):
    ranges = [row_range(H, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == H
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0
    sizes = [r1 - r0 for r0, r1 in ranges]
    assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, H, W, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
        import rti_oracle as o

        lu, lv = o.synth_dirs(20, 1)
        I = o.synth_intensities(H, W, lu, lv, seed=4)  # every rank holds the same image, fits its rows
        pv = o.pinv_shared("ptm", lu, lv)
        r0, r1 = row_range(H, world, rank)
        local = torch.as_tensor(o.fit_shared(I[:, r0:r1], pv).reshape(r1 - r0, W, 6))
        full = gather_rows(local, H)
        # the gathered map must be exactly the row blocks every rank fitted, in row order
        ref = np.concatenate([o.fit_shared(I[:, a:b], pv).reshape(b - a, W, 6)
                              for a, b in (row_range(H, world, r) for r in range(world))])
        q.put((rank, bool(np.array_equal(full.numpy(), ref)), tuple(full.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("H,W", [(9, 5), (16, 8)])
def test_gather_rows_two_ranks(H, W):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, shape in results:
        assert ok and shape == (H, W, 6), (rank, shape)


def _pipelined_worker(rank, world, port, H, W, chunks, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full_ref = torch.arange(H * W * 6, dtype=torch.float32).reshape(H, W, 6)
        r0, r1 = row_range(H, world, rank)
        calls = []

        def produce(c0, c1):  # stands in for one fit launch per row chunk
            calls.append((c0, c1))
            return full_ref[r0 + c0: r0 + c1].clone()

        full = gather_rows_pipelined(produce, r1 - r0, H, (W, 6), torch.float32, torch.device("cpu"), chunks=chunks)
        covered = sorted(calls) == calls and sum(b - a for a, b in calls) == r1 - r0
        ok = bool(torch.equal(full, full_ref))
        # with a caller-kept staging dict the second call reuses the first call's buffers (no allocation)
        staging = {}
        for it in range(2):
            out = gather_rows_pipelined(produce, r1 - r0, H, (W, 6), torch.float32, torch.device("cpu"),
                                        chunks=chunks, staging=staging)
            ok = ok and bool(torch.equal(out, full_ref))
            ptrs = {k: v.data_ptr() for k, v in staging.items()}
            if it == 0:
                first = ptrs
        ok = ok and ptrs == first
        q.put((rank, ok, covered))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("H,W,chunks,world", [(9, 5, 4, 2), (16, 8, 3, 2), (3, 4, 4, 2), (1, 3, 2, 2), (11, 2, 5, 3)])
def test_gather_rows_pipelined(H, W, chunks, world):
    """Chunked all-gather (overlapped with the per-chunk fit on GPUs) reassembles the exact map,
    including ranks with fewer rows than chunks and ranks with no rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, H, W, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, covered in results:
        assert ok and covered, rank


@pytest.mark.parametrize("H,world,chunks", [(2160, 8, 3), (2160, 4, 4), (40, 2, 4), (12, 3, 2)])
def test_cyclic_rows_partition(H, world, chunks):
    blocks = [b for r in range(world) for b in cyclic_rows(H, world, r, chunks)]
    assert sorted(blocks) == [(i * H // (world * chunks), (i + 1) * H // (world * chunks))
                              for i in range(world * chunks)]
    # chunk c of all ranks is one contiguous row range, rank-major: the in-place gather target
    for c in range(chunks):
        rows = [cyclic_rows(H, world, r, chunks)[c] for r in range(world)]
        assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
    with pytest.raises(ValueError):
        cyclic_rows(H + 1, world, 0, chunks)


def _cyclic_worker(rank, world, port, H, W, chunks, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full_ref = torch.arange(H * W * 6, dtype=torch.float32).reshape(H, W, 6)
        local = torch.cat([full_ref[a:b] for a, b in cyclic_rows(H, world, rank, chunks)])

        def produce(c0, c1):
            return local[c0:c1].clone()

        out = torch.full((H, W, 6), -1.0)
        full = gather_rows_pipelined(produce, local.shape[0], H, (W, 6), torch.float32, torch.device("cpu"),
                                     chunks=chunks, partition="cyclic", out=out)
        q.put((rank, bool(torch.equal(full, full_ref)) and full is out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("H,W,chunks,world", [(16, 3, 4, 2), (12, 2, 2, 3)])
def test_gather_rows_pipelined_cyclic(H, W, chunks, world):
    """Block-cyclic rows: every chunk's all-gather lands in place in the caller's map."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cyclic_worker, args=(r, world, port, H, W, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in results:
        assert ok, rank


def _bench_plan(args):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                       timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [2, 4])
def test_bench_spawns_ranks_strong_scaling(gpus):
    """bench.py --gpus N re-launches itself under torch.distributed.run with N ranks; by default each
    rank gets H/N rows of the same image (strong scaling)."""
    line = _bench_plan(["--gpus", str(gpus), "--plan", "--config", "c3"])
    assert line["n_gpus"] == gpus and line["scaling"] == "strong"
    assert line["config"]["H"] == 2160 and line["config"]["H_per_rank"] == 2160 // gpus
    assert line["config"]["rows_per_rank"] == [[r * 2160 // gpus, (r + 1) * 2160 // gpus] for r in range(gpus)]


def test_bench_weak_option():
    line = _bench_plan(["--gpus", "2", "--plan", "--weak"])
    assert line["scaling"] == "weak" and line["config"]["H_per_rank"] == 2160 and line["config"]["H"] == 4320


def _channels_worker(rank, world, port, H, W, C, chunks, partition, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rti.parallel import gather_evals, local_to_global_row

        full_ref = torch.arange(C * H * W * 6, dtype=torch.float32).reshape(C, H, W, 6)
        if partition == "cyclic":
            local = torch.cat([full_ref[:, a:b] for a, b in cyclic_rows(H, world, rank, chunks)], dim=1)
        else:
            r0, r1 = row_range(H, world, rank)
            local = full_ref[:, r0:r1].clone()
        origins = []

        def produce(c0, c1):  # every channel's rows of the chunk, as one fit launch produces them
            origins.append(local_to_global_row(H, world, rank, chunks, partition, c0))
            return local[:, c0:c1].clone()

        full = gather_rows_pipelined(produce, local.shape[1], H, (W, 6), torch.float32, torch.device("cpu"),
                                     chunks=chunks, partition=partition, channels=C)
        # the global row origin of every produced chunk: its first row's index in the whole image
        want = [int(local[0, c0, 0, 0]) // (W * 6) for c0 in
                ([j * (local.shape[1] // chunks) for j in range(chunks)] if partition == "cyclic" else
                 [row_range(local.shape[1], min(chunks, local.shape[1]) or 1, j)[0]
                  for j in range(max(1, min(chunks, local.shape[1])))])] if local.shape[1] else []
        ok_origins = origins == want[:len(origins)]
        # relit rows [E, h, W] -> whole [E, H, W] images
        E = 3
        img_ref = torch.arange(E * H * W, dtype=torch.float32).reshape(E, H, W)
        r0, r1 = row_range(H, world, rank)
        imgs = gather_evals(img_ref[:, r0:r1], H)
        q.put((rank, bool(torch.equal(full, full_ref)), ok_origins, bool(torch.equal(imgs, img_ref))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("H,W,C,chunks,world,partition", [(16, 3, 3, 4, 2, "block"), (11, 2, 3, 3, 3, "block"),
                                                          (12, 2, 3, 2, 3, "cyclic"), (16, 4, 2, 4, 2, "cyclic")])
def test_gather_rows_pipelined_channels(H, W, C, chunks, world, partition):
    """C > 1 (RGB / HSH-16 maps): each chunk's rows of every channel gathered into the
    [C, H, W, k] map (even and ragged block partitions, block-cyclic in place); the global row origin a
    per-pixel chunk needs (analysis.py:228); relit row blocks reassembled into whole images."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_channels_worker, args=(r, world, port, H, W, C, chunks, partition, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, ok_origins, ok_imgs in results:
        assert ok and ok_origins and ok_imgs, (rank, ok, ok_origins, ok_imgs)
