"""Row-block tiling of the shared fit over ranks (one process per GPU).

The fit is embarrassingly parallel over pixels: rank r of G fits its row blocks of the image
with the replicated k×N pseudo-inverse, and the only exchange is an all-gather that reassembles
the coefficient maps (``torch.distributed`` with backend "nccl" = RCCL over xGMI; "gloo" on CPU
for tests).  The reference has no parallelism of any kind.

Two row partitions:
  * block  — rank r holds rows row_range(H, G, r) = [r·H/G, (r+1)·H/G).  When G divides H one
    ``all_gather_into_tensor`` writes every rank's block straight into the [H, ...] map.
  * cyclic — the image is cut into G·chunks blocks of H/(G·chunks) rows and block b belongs to
    rank b mod G (cyclic_rows).  Chunk c of every rank then covers the contiguous rows
    [c·G·hc, (c+1)·G·hc), so the overlapped pipeline gathers each chunk in place: no staging
    copy at all.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L
from . import api


def row_range(H, world, rank):
    """Contiguous row block of `rank`: sizes differ by at most one row."""
    base, rem = divmod(H, world)
    r0 = rank * base + min(rank, rem)
    return r0, r0 + base + (1 if rank < rem else 0)


def cyclic_rows(H, world, rank, chunks):
    """Row blocks (r0, r1) of `rank` under the block-cyclic partition (H divisible by world·chunks):
    block b = rows [b·hc, (b+1)·hc), hc = H/(world·chunks), belongs to rank b mod world."""
    if H % (world * chunks):
        raise ValueError(f"cyclic partition needs H={H} divisible by world*chunks={world * chunks}")
    hc = H // (world * chunks)
    return [((c * world + rank) * hc, (c * world + rank + 1) * hc) for c in range(chunks)]


def _nccl(group):
    return dist.get_backend(group) == "nccl"


def gather_rows(local, H, group=None, out=None):
    """All-gather row blocks [h_r, ...] (block partition) from every rank into the full [H, ...] map.

    G | H: one all_gather_into_tensor (RCCL) lands every block in place, into ``out`` if given.
    Otherwise blocks differ by one row: they are padded to the largest block and trimmed.
    gloo (CPU tests) moves host tensors."""
    world = dist.get_world_size(group)
    trail = tuple(local.shape[1:])
    if H % world == 0:
        if local.shape[0] != H // world:
            raise ValueError(f"local block has {local.shape[0]} rows, expected {H // world}")
        full = out if out is not None else torch.empty((H,) + trail, dtype=local.dtype, device=local.device)
        if _nccl(group):
            dist.all_gather_into_tensor(full, local.contiguous(), group=group)
            return full
        host = full if full.device.type == "cpu" else torch.empty(full.shape, dtype=full.dtype)
        dist.all_gather(list(host.split(H // world)), local.contiguous().cpu(), group=group)
        if host is not full:
            full.copy_(host)
        return full
    rows = [row_range(H, world, r) for r in range(world)]
    hmax = max(r1 - r0 for r0, r1 in rows)
    pad = torch.zeros((hmax,) + trail, dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    if _nccl(group):
        buf = torch.empty((world * hmax,) + trail, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(buf, pad, group=group)
        parts = buf.split(hmax)
    else:
        host = pad.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
    full = out if out is not None else torch.empty((H,) + trail, dtype=local.dtype, device=local.device)
    for p, (r0, r1) in zip(parts, rows):
        full[r0:r1] = p[: r1 - r0]
    return full


def fit_rowtiled(I_rows, lu, lv, H, basis="ptm", rcond=None, gather=True, group=None, **kw):
    """Fit this rank's row block I_rows [N, h_r, W] and optionally all-gather the maps.

    Returns the full [H, W, k] coefficient map when gather=True, else the local block."""
    coef = api.fit(I_rows, lu, lv, basis=basis, mode="shared", rcond=rcond, layout="pixel", **kw)
    if not gather:
        return coef
    return gather_rows(coef, H, group=group)


def gather_rows_pipelined(produce, h_local, H, trail, dtype, device, chunks=4, group=None, partition="block",
                          out=None):
    """All-gather a row-tiled map while it is being produced (overlap the coefficient
    all-gather with fitting).

    ``produce(c0, c1)`` enqueues (on the current stream) and returns rows [c0, c1) of this rank's
    local rows, contiguous.  The local rows are cut into ``chunks`` row chunks; chunk c's all-gather is
    issued asynchronously right after chunk c is produced, so with backend "nccl" (RCCL over xGMI) it
    runs on the communicator's stream — ordered after the kernel that produced it — while the current
    stream produces chunk c + 1.

    partition="cyclic": this rank's local rows are its cyclic_rows(H, G, r, chunks) blocks in order;
    every chunk is gathered straight into its place in the [H, *trail] map.
    partition="block": local rows = row_range(H, G, r); with G | H and chunks | H/G each chunk is
    gathered into a staging buffer and moved into place by one strided copy; other shapes pad.
    Returns the full [H, *trail] map."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    nccl = _nccl(group)
    full = out if out is not None else torch.empty((H,) + tuple(trail), dtype=dtype, device=device)
    if partition == "cyclic":
        blocks = cyclic_rows(H, world, rank, chunks)
        hc = blocks[0][1] - blocks[0][0]
        if h_local != hc * chunks:
            raise ValueError(f"rank {rank} holds {h_local} rows, the cyclic partition gives {hc * chunks}")
        pending = []
        for c in range(chunks):
            part = produce(c * hc, (c + 1) * hc)
            dst = full[c * world * hc:(c + 1) * world * hc]
            if nccl:
                pending.append(dist.all_gather_into_tensor(dst, part, group=group, async_op=True))
            else:
                host = [torch.empty((hc,) + tuple(trail), dtype=dtype) for _ in range(world)]
                pending.append((dist.all_gather(host, part.cpu(), group=group, async_op=True), host, dst))
        for p in pending:
            if nccl:
                p.wait()
            else:
                work, host, dst = p
                work.wait()
                dst.copy_(torch.cat(host))
        return full
    if partition != "block":
        raise ValueError(f"unknown partition {partition!r} (expected 'block' or 'cyclic')")
    rows = [row_range(H, world, r) for r in range(world)]
    if rows[rank][1] - rows[rank][0] != h_local:
        raise ValueError(f"rank {rank} holds {h_local} rows, row_range gives {rows[rank]}")
    hmax = max(r1 - r0 for r0, r1 in rows)
    chunks = max(1, min(chunks, hmax))
    even = H % world == 0 and (H // world) % chunks == 0
    cmax = -(-hmax // chunks)
    pending = []
    for c in range(chunks):
        c0, c1 = row_range(h_local, chunks, c)
        if even:
            part = produce(c0, c1)
        else:
            part = torch.zeros((cmax,) + tuple(trail), dtype=dtype, device=device)
            if c1 > c0:
                part[: c1 - c0] = produce(c0, c1)
        if nccl:
            buf = torch.empty((world,) + tuple(part.shape), dtype=dtype, device=device)
            pending.append((dist.all_gather_into_tensor(buf.view((-1,) + tuple(trail)), part, group=group,
                                                        async_op=True), buf))
        else:
            host = part.cpu()
            bufs = [torch.empty_like(host) for _ in range(world)]
            pending.append((dist.all_gather(bufs, host, group=group, async_op=True), bufs))
    hb = H // world if even else None
    for c, (work, parts) in enumerate(pending):
        work.wait()
        if not nccl:
            parts = torch.stack(parts).to(device)
        if even:  # one strided copy: rank r's chunk c -> rows r·hb + [c0, c1)
            c0, c1 = row_range(hb, chunks, c)
            full.view((world, hb) + tuple(trail))[:, c0:c1] = parts
            continue
        for r in range(world):
            h_r = rows[r][1] - rows[r][0]
            c0, c1 = row_range(h_r, chunks, c)
            full[rows[r][0] + c0:rows[r][0] + c1] = parts[r][: c1 - c0].to(device)
    return full


class RowTiledFitter:
    """Row-tiled shared fit of this rank's rows with the all-gather of each row chunk overlapped with
    the fit of the next (one rti_fit_shared launch per chunk on the current stream).  The pseudo-
    inverse, the local coefficient rows and the full map are allocated once; ``__call__`` returns the
    full [H, W, k] map (the same tensor every call).

    I_rows: this rank's CUDA light-major rows [N, h, W] (block partition: rows row_range(H, G, r);
    cyclic: its cyclic_rows(H, G, r, chunks) blocks in order)."""

    def __init__(self, I_rows, lu, lv, H, basis="ptm", rcond=None, chunks=4, group=None, kernel="auto",
                 partition="block"):
        api._require_cuda(I_rows, "I_rows")
        self.N, self.h, self.W = I_rows.shape
        self.H, self.chunks, self.group, self.partition = H, chunks, group, partition
        b = api.basis_id(basis)
        self.k = api.basis_terms(b)
        dev = I_rows.device
        self.pinv = torch.as_tensor(api.pinv(lu, lv, basis, rcond=rcond).astype(np.float32), device=dev)
        self.I = I_rows.contiguous()
        self.coef = torch.empty((self.h, self.W, self.k), dtype=torch.float32, device=dev)
        self.full = torch.empty((H, self.W, self.k), dtype=torch.float32, device=dev)
        self.kern = api._KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
        self.dt = api._IN_DTYPES[self.I.dtype]

    def _produce(self, c0, c1):
        W, k, N, es = self.W, self.k, self.N, self.I.element_size()
        st = L.lib().rti_fit_shared(api._vp(self.pinv), k, N, self.I.data_ptr() + c0 * W * es, self.dt,
                                    (c1 - c0) * W, 1, self.h * W, 0, self.coef.data_ptr() + c0 * W * k * 4,
                                    L.RTI_COEF_PIXEL_MAJOR, 0, self.kern, api._stream_of(self.I))
        L.check(st, "rti_fit_shared")
        return self.coef[c0:c1]

    def __call__(self):
        return gather_rows_pipelined(self._produce, self.h, self.H, (self.W, self.k), torch.float32,
                                     self.I.device, chunks=self.chunks, group=self.group,
                                     partition=self.partition, out=self.full)


def fit_rowtiled_overlapped(I_rows, lu, lv, H, basis="ptm", rcond=None, chunks=4, group=None, kernel="auto",
                            partition="block"):
    """One-shot form of RowTiledFitter: returns the full [H, W, k] map on every rank."""
    return RowTiledFitter(I_rows, lu, lv, H, basis=basis, rcond=rcond, chunks=chunks, group=group, kernel=kernel,
                          partition=partition)()
