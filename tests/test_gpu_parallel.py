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
                                              (2, "64x96", ["--weak"])])
def test_bench_multi_rank_end_to_end_parity(cuda, gpus, shape, extra):
    """bench.py --gpus N (ranks sharing cuda:0 over gloo): the strong-scaling line, the all-gather legs and
    the overlapped row-chunked fit whose gathered map (block-cyclic rows generated per rank) rank 0 checks
    block by block against the oracle (e2e_parity)."""
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
