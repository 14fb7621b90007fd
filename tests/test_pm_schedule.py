"""CPU check of the streaming pixel-major fit's schedule (csrc/rti_fit_pm.hip, fit_pm_stream): the
kernel's scalar bookkeeping restated in Python and run for every wave of real launch shapes.  It checks
what a wrong count would turn into a silent race or an out-of-range access on the GPU: every DMA reads
inside its channel and lands in a ring slot whose bytes were consumed, every group's wait count equals
the vector-memory ops issued after the DMA it needs, and the groups of all waves cover every pixel of
every channel exactly once."""
import math

import pytest

WAITS = (0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48)


def plan(N, P, C, W, ring, U=1, cus=256):
    U = 16 // math.gcd(N, 16) * U  # units of whole KiB (launch_stream_t)
    nu = -(-P // (16 * U))
    tu = nu * C
    wgs = -(-tu // W)
    grid = min(wgs, cus)
    return U, nu, tu, grid * W


def simulate_wave(gw, GW, N, P, C, U, nu, tu, ring, S, contig):
    GBY = 64 * N
    UB = U * GBY
    assert UB % 1024 == 0
    cbytes = P * N * 4
    slots = ring // 1024
    if contig:
        per = -(-tu // GW)
        u0, ustep = gw * per, 1
        nk = 0 if u0 >= tu else min(per, tu - u0)
    else:
        u0, ustep = gw, GW
        nk = 0 if gw >= tu else (tu - 1 - gw) // GW + 1
    if nk == 0:
        return []
    ng, dt = nk * U, -(-(nk * UB) // 1024)
    ops = []  # ("d", d) / ("s", j)
    cur = {"cd": u0 // nu, "ud": u0 % nu, "inb": 0, "wslot": 0}
    consumed = 0
    dma_units = {}  # d -> {(channel, unit)} its lanes read

    def nxt(c, u):
        u += ustep
        while u >= nu:
            u -= nu
            c += 1
        return c, u

    def issue(d):
        assert cur["cd"] < C
        c2, u2 = nxt(cur["cd"], cur["ud"])
        units = set()
        for lane in range(64):
            lb = 16 * lane
            here = lb < UB - cur["inb"]
            off = cur["ud"] * UB + cur["inb"] + lb if here else u2 * UB + (lb - (UB - cur["inb"]))
            cc = cur["cd"] if here else (c2 if c2 < C else cur["cd"])
            if here or c2 < C:
                units.add((cc, off // UB))
            off = off if off + 16 <= cbytes else cbytes - 16
            assert 0 <= off <= cbytes - 16 and 0 <= cc < C
        # the ring bytes this DMA overwrites must be consumed: stream bytes [1024d - ring, 1024(d+1) - ring)
        assert 1024 * (d + 1) - ring <= consumed, (d, consumed)
        assert cur["wslot"] == (1024 * d) % ring
        dma_units[d] = units
        ops.append(("d", d))
        cur["wslot"] = (cur["wslot"] + 1024) % ring
        cur["inb"] += 1024
        if cur["inb"] >= UB:
            cur["inb"] -= UB
            cur["cd"], cur["ud"] = c2, u2

    issued = min(dt, slots)
    for d in range(issued):
        issue(d)
    cg, ug, gi = u0 // nu, u0 % nu, 0
    gd = -1
    covered = []
    for j in range(ng):
        end = GBY * (j + 1)
        dn = (end + 1023) // 1024 - 1
        while ((GBY * (gd + 1) + ring) >> 10) < dn + 1:
            gd += 1
        n = (issued - 1 - dn) + S * (j - 1 - gd)
        # exact: the ops issued after DMA dn
        idx = ops.index(("d", dn))
        assert n == len(ops) - 1 - idx, (j, n, len(ops) - 1 - idx)
        m = max(w for w in WAITS if w <= min(n, 63))
        assert m <= n
        # the group's bytes come from DMAs whose lanes read its own unit
        first = GBY * j // 1024
        for d in range(first, dn + 1):
            assert (cg, ug) in dma_units[d], (j, d)
        covered.append((cg, (ug * U + gi) * 16))
        for _ in range(S):
            ops.append(("s", j))
        consumed = end
        lim = min(dt, (end + ring) >> 10)
        while issued < lim:
            issue(issued)
            issued += 1
        gi += 1
        if gi == U:
            gi = 0
            ug += ustep
            while ug >= nu:
                ug -= nu
                cg += 1
    assert issued == dt
    return covered


@pytest.mark.parametrize("N,P,C,W,K_S", [(100, 3840 * 2160, 1, 8, 2), (200, 3840 * 2160, 3, 8, 1), (200, 3840 * 2160, 3, 4, 1),
                                          (50, 1920 * 1080, 1, 8, 2), (20, 256 * 256, 1, 8, 4), (33, 2384, 3, 8, 2),
                                          (17, 4100, 2, 3, 4), (256, 1000, 2, 3, 1), (100, 5000, 2, 8, 2), (16, 300, 3, 8, 2)])
@pytest.mark.parametrize("contig", [0, 1])
@pytest.mark.parametrize("U", [1, 2])
def test_stream_schedule(N, P, C, W, K_S, contig, U):
    op = 16 * (-(-N // 16) * 16) * 4
    ring = ((160 * 1024 - op) // W) >> 10 << 10
    if ring < 64 * N + 1024:
        pytest.skip("no ring")
    U, nu, tu, GW = plan(N, P, C, W, ring, U)
    waves = range(GW) if GW * tu < 2_000_000 else sorted({0, 1, GW // 2, GW - 2, GW - 1})
    seen = set()
    for gw in waves:
        for c, p0 in simulate_wave(gw, GW, N, P, C, U, nu, tu, ring, K_S, contig):
            assert (c, p0) not in seen
            seen.add((c, p0))
    if len(waves) == GW:
        want = {(c, 16 * g) for c in range(C) for g in range(nu * U)}
        assert seen == want  # every group of every channel (groups past P are computed and never stored)
        assert all(p0 < nu * U * 16 for _, p0 in seen) and math.ceil(P / 16) <= nu * U
