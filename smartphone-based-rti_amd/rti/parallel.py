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
                          out=None, channels=None, staging=None):
    """All-gather a row-tiled map while it is being produced (overlap the coefficient
    all-gather with fitting).

    ``produce(c0, c1)`` enqueues (on the current stream) and returns rows [c0, c1) of this rank's
    local rows, contiguous.  The local rows are cut into ``chunks`` row chunks; chunk c's all-gather is
    issued asynchronously right after chunk c is produced, so with backend "nccl" (RCCL over xGMI) it
    runs on the communicator's stream — ordered after the kernel that produced it — while the current
    stream produces chunk c + 1.

    channels=C: ``produce`` returns [C, c1 - c0, *trail] (every channel's rows of the chunk, one fit
    launch) and the map is [C, H, *trail]; each channel's rows are gathered by their own collective.

    partition="cyclic": this rank's local rows are its cyclic_rows(H, G, r, chunks) blocks in order;
    every chunk is gathered straight into its place in the [H, *trail] map.
    partition="block": local rows = row_range(H, G, r); with G | H and chunks | H/G each chunk is
    gathered into a staging buffer and moved into place by one strided copy; other shapes pad.
    staging: a dict the caller keeps across calls (RowTiledFitter does); the block partition's staging and
    pad buffers live there, so only the first call allocates.
    Returns the full [H, *trail] (or [C, H, *trail]) map."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    nccl = _nccl(group)
    trail = tuple(trail)
    C = 1 if channels is None else int(channels)
    lead = () if channels is None else (C,)
    full = out if out is not None else torch.empty(lead + (H,) + trail, dtype=dtype, device=device)
    fullc = full.unsqueeze(0) if channels is None else full  # [C, H, *trail]

    def parts_of(part):  # the chunk's rows per channel
        return [part] if channels is None else [part[c] for c in range(C)]

    if partition == "cyclic":
        blocks = cyclic_rows(H, world, rank, chunks)
        hc = blocks[0][1] - blocks[0][0]
        if h_local != hc * chunks:
            raise ValueError(f"rank {rank} holds {h_local} rows, the cyclic partition gives {hc * chunks}")
        pending = []
        for j in range(chunks):
            part = produce(j * hc, (j + 1) * hc)
            for c, pc in enumerate(parts_of(part)):
                dst = fullc[c][j * world * hc:(j + 1) * world * hc]
                if nccl:
                    pending.append(dist.all_gather_into_tensor(dst, pc.contiguous(), group=group, async_op=True))
                else:
                    host = [torch.empty((hc,) + trail, dtype=dtype) for _ in range(world)]
                    pending.append((dist.all_gather(host, pc.cpu(), group=group, async_op=True), host, dst))
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

    def staged(key, shape, zero=False):
        """A device buffer for this call's chunk `key`: from `staging` (allocated on its first call, reused
        after: the previous call's copies out of it are ordered before this call's collective on the stream)."""
        if staging is None:
            return (torch.zeros if zero else torch.empty)(shape, dtype=dtype, device=device)
        buf = staging.get(key)
        if buf is None or tuple(buf.shape) != tuple(shape) or buf.dtype != dtype:
            buf = staging[key] = (torch.zeros if zero else torch.empty)(shape, dtype=dtype, device=device)
        elif zero:
            buf.zero_()
        return buf

    pending = []
    for j in range(chunks):
        c0, c1 = row_range(h_local, chunks, j)
        if even:
            pcs = parts_of(produce(c0, c1))
        else:
            pad = staged(("pad", j), lead + (cmax,) + trail, zero=True)
            if c1 > c0:
                pad.narrow(len(lead), 0, c1 - c0).copy_(produce(c0, c1))
            pcs = parts_of(pad)
        for c, part in enumerate(pcs):
            part = part.contiguous()
            if nccl:
                buf = staged(("gather", c, j), (world,) + tuple(part.shape))
                pending.append((c, j, dist.all_gather_into_tensor(buf.view((-1,) + trail), part, group=group,
                                                                  async_op=True), buf))
            else:
                host = part.cpu()
                bufs = [torch.empty_like(host) for _ in range(world)]
                pending.append((c, j, dist.all_gather(bufs, host, group=group, async_op=True), bufs))
    hb = H // world if even else None
    for c, j, work, parts in pending:
        work.wait()
        if not nccl:
            parts = torch.stack(parts).to(device)
        if even:  # one strided copy: rank r's chunk j -> rows r·hb + [c0, c1)
            c0, c1 = row_range(hb, chunks, j)
            fullc[c].view((world, hb) + trail)[:, c0:c1] = parts
            continue
        for r in range(world):
            h_r = rows[r][1] - rows[r][0]
            c0, c1 = row_range(h_r, chunks, j)
            fullc[c][rows[r][0] + c0:rows[r][0] + c1] = parts[r][: c1 - c0].to(device)
    return full


def local_to_global_row(H, world, rank, chunks, partition, c0):
    """Global image row of local row c0 at the start of a produced chunk (the row origin a per-pixel
    fit needs: analysis.py:228 takes p = (x, y, 0) in whole-image indices)."""
    if partition == "cyclic":
        blocks = cyclic_rows(H, world, rank, chunks)
        hc = blocks[0][1] - blocks[0][0]
        j, off = divmod(c0, hc)
        return blocks[j][0] + off
    return row_range(H, world, rank)[0] + c0


class RowTiledFitter:
    """Row-tiled fit of this rank's rows with the all-gather of each row chunk overlapped with the fit of
    the next (one fit launch per chunk, all channels, on the current stream).  The operator, the local
    coefficient rows and the full map are allocated once; ``__call__`` returns the full map (the same
    tensor every call): [H, W, k] for one channel, [C, H, W, k] for C (every pixel is
    independent, the only exchange is the coefficient all-gather).

    I_rows: this rank's CUDA rows (block partition: rows row_range(H, G, r); cyclic: its
    cyclic_rows(H, G, r, chunks) blocks in order), in any form rti.fit takes:
      * mode="shared", stack="light": light-major [N, h, W] or [C, N, h, W], fp32 / int32 / uint8; 8-bit
        stacks run the split-fp16 matrix-core fit (rti_fit_shared_h16, rti.fit's AUTO) when W is a
        multiple of 16, else rti_fit_shared;
      * mode="shared", stack="pixel": the reference's pixel-major [h, W, N] or [C, h, W, N]
        (analysis.py:217-219), fitted in place by rti_fit_shared_pm;
      * mode="perpixel" (PTM-6): cams [N, 3] and light-major [N, h, W]; each chunk's light vectors use its
        rows' GLOBAL image indices (rti_fit_perpixel_cam with the chunk's row origin, analysis.py:228), so
        the gathered map equals the whole-image fit; coef_dtype fp32 or fp64."""

    def __init__(self, I_rows, lu=None, lv=None, H=None, basis="ptm", rcond=None, chunks=4, group=None,
                 kernel="auto", partition="block", stack="light", mode="shared", cams=None, origin=(0.0, 0.0),
                 coef_dtype=torch.float32):
        api._require_cuda(I_rows, "I_rows")
        if H is None:
            raise ValueError("H (the whole image's rows) is required")
        if mode not in ("shared", "perpixel"):
            raise ValueError(f"unknown mode {mode!r}")
        if stack not in ("light", "pixel"):
            raise ValueError(f"unknown stack layout {stack!r}")
        self.H, self.chunks, self.group, self.partition = H, chunks, group, partition
        self.mode, self.stack, self.origin = mode, stack, (float(origin[0]), float(origin[1]))
        dev = I_rows.device
        self.I = I_rows.contiguous()
        if mode == "perpixel":
            if api.basis_id(basis) != L.RTI_BASIS_PTM6 or stack != "light" or self.I.dim() != 3:
                raise ValueError("per-pixel row tiling: PTM-6, light-major [N, h, W] rows and cams")
            self.C, (self.N, self.h, self.W) = 1, self.I.shape
            self.k = 6
            self.cdt = api._COEF_DTYPES.get(coef_dtype)
            if self.cdt is None:
                raise ValueError("coef_dtype must be torch.float32 or torch.float64")
            cams_np = np.asarray(cams.detach().cpu() if torch.is_tensor(cams) else cams, np.float64)
            self.cams = torch.as_tensor(cams_np, device=dev).contiguous()
            if self.cams.shape != (self.N, 3):
                raise ValueError(f"cams must be [{self.N}, 3]")
            self.rc = -1.0 if rcond is None else float(rcond)
            self.dtype = coef_dtype
        else:
            if lu is None or lv is None:
                raise ValueError("shared mode needs lu and lv")
            if stack == "light":
                x = self.I if self.I.dim() == 4 else self.I.unsqueeze(0)
                self.C, self.N, self.h, self.W = x.shape
            else:
                x = self.I if self.I.dim() == 4 else self.I.unsqueeze(0)
                self.C, self.h, self.W, self.N = x.shape
            b = api.basis_id(basis)
            self.k = api.basis_terms(b)
            pv = api.pinv(lu, lv, basis, rcond=rcond)
            if pv.shape[1] != self.N:
                raise ValueError(f"{pv.shape[1]} light directions for {self.N} intensity planes")
            self.pinv = torch.as_tensor(pv.astype(np.float32), device=dev)
            self.dtype = torch.float32
            # 8-bit matrix-core fits (rti.fit's AUTO for uint8 light-major stacks, or asked for by name): the
            # split-fp16 operator (rti_fit_shared_h16) or the int8 fixed-point one (rti_fit_shared_q8)
            self.u8, self.u8_op = None, None
            mk = "h16" if kernel == "auto" else kernel
            if isinstance(kernel, str) and kernel not in api._KERNELS and kernel not in ("h16", "q8"):
                raise ValueError(f"unknown kernel {kernel!r}")
            if mk in ("h16", "q8"):
                maxn = (L.lib().rti_fit_shared_h16_max_lights if mk == "h16" else
                        L.lib().rti_fit_shared_q8_max_lights)()
                ok = (stack == "light" and self.I.dtype == torch.uint8 and self.W % 16 == 0 and self.k in (6, 9, 16)
                      and self.N <= int(maxn) and np.isfinite(pv).all() and self.I.data_ptr() % 16 == 0)
                if ok:
                    self.u8 = mk
                    self.u8_op = torch.as_tensor(api.h16_operator(pv) if mk == "h16" else api.q8_operator(pv),
                                                 device=dev)
                elif kernel in ("h16", "q8"):
                    raise NotImplementedError(f"kernel={kernel!r} needs a light-major uint8 stack, W % 16 == 0, "
                                              f"k in (6, 9, 16), N <= {int(maxn)} and a finite pseudo-inverse")
            # every other selector (string or integer kernel word) goes to rti_fit_shared / rti_fit_shared_pm
            # unchanged: the C entries refuse bits they do not document
            self.kern = 0 if mk in ("h16", "q8") else (api._KERNELS[kernel] if isinstance(kernel, str)
                                                       else int(kernel))
        self.dt = api._IN_DTYPES[self.I.dtype]
        self.coef = torch.empty((self.C, self.h, self.W, self.k), dtype=self.dtype, device=dev)
        lead = (self.C,) if self.C > 1 or self.I.dim() == 4 else ()
        self.full = torch.empty(lead + (H, self.W, self.k), dtype=self.dtype, device=dev)
        self.channels = self.C if lead else None
        self._staging = {}  # block-partition gather/pad buffers, allocated by the first call only

    def _produce(self, c0, c1):
        W, k, N, C, h = self.W, self.k, self.N, self.C, self.h
        es, ces = self.I.element_size(), self.coef.element_size()
        P = (c1 - c0) * W
        s = api._stream_of(self.I)
        ocs = h * W * k
        dst = self.coef.data_ptr() + c0 * W * k * ces
        lib = L.lib()
        if self.mode == "perpixel":
            world, rank = dist.get_world_size(self.group), dist.get_rank(self.group)
            y0 = local_to_global_row(self.H, world, rank, self.chunks, self.partition, c0)
            st = lib.rti_fit_perpixel_cam(api._vp(self.cams), N, self.I.data_ptr() + c0 * W * es, self.dt, c1 - c0,
                                          W, h * W, self.origin[0], self.origin[1] + y0, self.rc, dst, self.cdt,
                                          L.RTI_COEF_PIXEL_MAJOR, s)
            L.check(st, "rti_fit_perpixel_cam")
        elif self.stack == "pixel":
            st = lib.rti_fit_shared_pm(api._vp(self.pinv), k, N, self.I.data_ptr() + c0 * W * N * es, self.dt, P, C,
                                       N, h * W * N, dst, L.RTI_COEF_PIXEL_MAJOR, ocs, self.kern, s)
            L.check(st, "rti_fit_shared_pm")
        elif self.u8 is not None:
            fn = lib.rti_fit_shared_h16 if self.u8 == "h16" else lib.rti_fit_shared_q8
            st = fn(api._vp(self.u8_op), k, N, self.I.data_ptr() + c0 * W, P, C, h * W, N * h * W,
                    dst, L.RTI_COEF_PIXEL_MAJOR, ocs, 0, s)
            L.check(st, f"rti_fit_shared_{self.u8}")
        else:
            st = lib.rti_fit_shared(api._vp(self.pinv), k, N, self.I.data_ptr() + c0 * W * es, self.dt, P, C, h * W,
                                    N * h * W, dst, L.RTI_COEF_PIXEL_MAJOR, ocs, self.kern, s)
            L.check(st, "rti_fit_shared")
        return self.coef[:, c0:c1] if self.channels else self.coef[0, c0:c1]

    def __call__(self):
        return gather_rows_pipelined(self._produce, self.h, self.H, (self.W, self.k), self.dtype,
                                     self.I.device, chunks=self.chunks, group=self.group,
                                     partition=self.partition, out=self.full, channels=self.channels,
                                     staging=self._staging)


def fit_rowtiled_overlapped(I_rows, lu=None, lv=None, H=None, basis="ptm", rcond=None, chunks=4, group=None,
                            kernel="auto", partition="block", **kw):
    """One-shot form of RowTiledFitter: returns the full map on every rank."""
    return RowTiledFitter(I_rows, lu, lv, H, basis=basis, rcond=rcond, chunks=chunks, group=group, kernel=kernel,
                          partition=partition, **kw)()


def gather_evals(local, H, group=None):
    """[E, h_r, W] relit rows of every rank (block partition) -> the whole [E, H, W] images: the rows are
    gathered as [h_r, E, W] (rows outermost, so row blocks land in order) and viewed back."""
    full = gather_rows(local.permute(1, 0, 2).contiguous(), H, group=group)  # [H, E, W]
    return full.permute(1, 0, 2)


def relight_rowtiled(coef_rows, lu, lv, H, basis="ptm", *, gather=False, group=None, out_dtype=torch.float32):
    """relight is row-shardable.  Every rank evaluates its own coefficient rows
    [h_r, W, k] (block partition) at the E directions (rti.relight, interactive_relighting.py:11-39 /
    analysis.py:300-315): no exchange.  gather=True assembles whole [E, H, W] images on every rank (a
    display), one all-gather."""
    img = api.relight(coef_rows, lu, lv, basis=basis, out_dtype=out_dtype)
    scalar = img.dim() == 2
    loc = img.unsqueeze(0) if scalar else img  # [E, h, W]
    if not gather:
        return img
    full = gather_evals(loc, H, group=group)
    return full[0] if scalar else full
