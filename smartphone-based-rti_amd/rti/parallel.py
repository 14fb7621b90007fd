"""Row-block tiling of the shared fit over ranks (one process per GPU).

The fit is embarrassingly parallel over pixels: rank r of G fits rows
[r·H/G, (r+1)·H/G) of the image with the replicated k×N pseudo-inverse, and
the only exchange is an all-gather that reassembles the coefficient maps
(``torch.distributed`` with backend "nccl" = RCCL over xGMI; "gloo" on CPU for
tests).  The reference has no parallelism of any kind.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import api


def row_range(H, world, rank):
    """Contiguous row block of `rank`: sizes differ by at most one row."""
    base, rem = divmod(H, world)
    r0 = rank * base + min(rank, rem)
    return r0, r0 + base + (1 if rank < rem else 0)


def gather_rows(local, H, group=None):
    """All-gather row blocks [h_r, ...] from every rank into the full [H, ...] map.

    Blocks are padded to the largest block so one all_gather_into_tensor (RCCL)
    moves them; gloo falls back to all_gather of equal-size tensors."""
    world = dist.get_world_size(group)
    rows = [row_range(H, world, r) for r in range(world)]
    hmax = max(r1 - r0 for r0, r1 in rows)
    pad = torch.zeros((hmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    if dist.get_backend(group) == "nccl":
        full = torch.empty((world * hmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(full, pad, group=group)
        parts = full.split(hmax)
    else:  # gloo: host tensors
        host = pad.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        parts = [p.to(local.device) for p in parts]
    return torch.cat([p[: r1 - r0] for p, (r0, r1) in zip(parts, rows)], dim=0)


def fit_rowtiled(I_rows, lu, lv, H, basis="ptm", rcond=None, gather=True, group=None, **kw):
    """Fit this rank's row block I_rows [N, h_r, W] and optionally all-gather the maps.

    Returns the full [H, W, k] coefficient map when gather=True, else the local block."""
    coef = api.fit(I_rows, lu, lv, basis=basis, mode="shared", rcond=rcond, layout="pixel", **kw)
    if not gather:
        return coef
    return gather_rows(coef, H, group=group)


def gather_rows_pipelined(produce, h_local, H, trail, dtype, device, chunks=4, group=None):
    """All-gather a row-tiled map while it is being produced (overlap the
    coefficient all-gather with fitting).

    ``produce(c0, c1)`` enqueues (on the current stream) and returns rows [c0, c1) of this
    rank's block.  The block is cut into ``chunks`` row chunks; chunk c's all-gather is issued
    asynchronously right after chunk c is produced, so with backend "nccl" (RCCL over xGMI)
    it runs on the communicator's stream — ordered after the kernel that produced it —
    while the current stream produces chunk c + 1.  ``trail``, ``dtype``, ``device``: the map's
    per-row shape and type (a rank may hold fewer rows than chunks, or none).  Returns the full
    [H, *trail] map."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rows = [row_range(H, world, r) for r in range(world)]
    if rows[rank][1] - rows[rank][0] != h_local:
        raise ValueError(f"rank {rank} holds {h_local} rows, row_range gives {rows[rank]}")
    hmax = max(r1 - r0 for r0, r1 in rows)
    chunks = max(1, min(chunks, hmax))
    cmax = -(-hmax // chunks)
    nccl = dist.get_backend(group) == "nccl"
    pending = []
    for c in range(chunks):
        c0, c1 = row_range(h_local, chunks, c)
        pad = torch.zeros((cmax,) + tuple(trail), dtype=dtype, device=device)
        if c1 > c0:
            pad[: c1 - c0] = produce(c0, c1)
        if nccl:
            buf = torch.empty((world * cmax,) + tuple(trail), dtype=dtype, device=device)
            work = dist.all_gather_into_tensor(buf, pad, group=group, async_op=True)
            pending.append((work, buf.split(cmax)))
        else:  # gloo: host tensors
            host = pad.cpu()
            bufs = [torch.empty_like(host) for _ in range(world)]
            work = dist.all_gather(bufs, host, group=group, async_op=True)
            pending.append((work, bufs))
    out_parts = [[None] * chunks for _ in range(world)]
    for c, (work, parts) in enumerate(pending):
        work.wait()
        for r in range(world):
            h_r = rows[r][1] - rows[r][0]
            c0, c1 = row_range(h_r, chunks, c)
            out_parts[r][c] = parts[r][: c1 - c0]
    full = torch.cat([p for r in range(world) for p in out_parts[r]], dim=0)
    return full.to(device)


def fit_rowtiled_overlapped(I_rows, lu, lv, H, basis="ptm", rcond=None, chunks=4, group=None, kernel="auto"):
    """Row-tiled shared fit with the all-gather of each row chunk overlapped with the fit of
    the next (one rti_fit_shared launch per chunk on the current stream).  I_rows: this rank's
    CUDA light-major block [N, h_r, W]; returns the full [H, W, k] map on every rank."""
    from . import _lib as L

    api._require_cuda(I_rows, "I_rows")
    N, h, W = I_rows.shape
    b = api.basis_id(basis)
    k = api.basis_terms(b)
    import numpy as np

    pinv = torch.as_tensor(api.pinv(lu, lv, basis, rcond=rcond).astype(np.float32), device=I_rows.device)
    I = I_rows.contiguous()
    coef = torch.empty((h, W, k), dtype=torch.float32, device=I.device)
    es = I.element_size()
    kern = api._KERNELS[kernel] if isinstance(kernel, str) else int(kernel)

    def produce(c0, c1):
        st = L.lib().rti_fit_shared(api._vp(pinv), k, N, I.data_ptr() + c0 * W * es, api._IN_DTYPES[I.dtype],
                                    (c1 - c0) * W, 1, h * W, 0, coef.data_ptr() + c0 * W * k * 4,
                                    L.RTI_COEF_PIXEL_MAJOR, 0, kern, api._stream_of(I))
        L.check(st, "rti_fit_shared")
        return coef[c0:c1]

    return gather_rows_pipelined(produce, h, H, (W, k), torch.float32, I.device, chunks=chunks, group=group)
