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
