"""CPU check of the column-group 4-D schedule (stem4d.hip
sk_stem4d_col_kernel): a step-by-step numpy emulation of the kernel's waves --
column groups of NB columns, positions, rows, the chains of one position (one
per column of the group, each chain's G0 row the next chain's A row), the LDS
B' double buffer by step parity, the round-wrap B' planes (one per chain), the
in-place G0 planes, the PF-rows-ahead fetch cursor -- in which every read of a
step sees memory as it was when the step began, an LDS write lands when the
step ends and a global write at the next full barrier.  A schedule that read
anything before it was written (a race between waves on the GPU) gives a
different K (unwritten memory is NaN); the emulated K must equal the C
oracle's full_dp (stem_kernel/stem_kernel.cpp:282-351) for several (n, m, W,
F, NB), including W at the host's limit m - F - 1 and groups cut short by n."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po

PF = 2


def group_positions(g, n, nb, F, pf=PF):
    """positions of column group g: its planes (i = j_hi - 1 down to 0),
    then bubbles up to F + PF"""
    j_hi = min((g + 1) * nb, n)
    return max(j_hi, F + pf)


class Pos:
    """stem4d.hip S4cPos: (group, offset in the group)"""
    def __init__(self):
        self.g, self.off = 0, 0

    def advance(self, W, n, nb, F, pf=PF):
        self.off += W
        while self.g * nb < n and self.off >= group_positions(self.g, n, nb, F, pf):
            self.off -= group_positions(self.g, n, nb, F, pf)
            self.g += 1

    def valid(self, n, nb):
        return self.g * nb < n

    def copy(self):
        q = Pos()
        q.g, q.off = self.g, self.off
        return q


def row_off(m, d2):
    return sum(((m + 1 - e) + 3) & ~3 for e in range(d2))


def bpdiag(seq, bpp):
    """stem4d_tables: prob(a, a+e) by diagonal, float (sk_api.cpp)."""
    L = len(seq)
    tri = {}
    k = 0
    for a in range(L):
        for b in range(a + 1, L):
            tri[(a, b)] = bpp[k]
            k += 1
    out = []
    for e in range(L):
        for a in range(L - e):
            out.append(np.float32(tri[(a, a + e)]) if e > 0 else np.float32(0.0))
    return np.array(out, np.float32)


def emulate(x, bx, y, by, W, F=1, nb=1, gap=0.8, stack=1.0, subst=0.5, bound=0.0, CPL=None, pf=PF,
            vis=None, zlead=None):
    """F: steps between full barriers -- a global store of step u is seen
    from the first multiple of F above u on; or, with vis, from step u + vis
    on (no full barriers: a wave's store is complete once it has waited for a
    load issued after it, PF steps later, and seen after the next barrier);
    LDS stores from the next step.  zlead: wave 0's round-wrap rows are
    loaded zlead steps before the step that uses them (by the staging waves),
    else with its own rows, PF steps ahead."""
    n, m = len(x), len(y)
    R = m + 1
    TW = 64 * (CPL or max(1, -(-(m + 1) // 64)))
    g = float(np.float32(gap))
    stk, sub = float(np.float32(stack)), float(np.float32(subst))
    bound = np.float32(bound)
    gpow = [1.0]
    for _ in range(max(n, m) + 2):
        gpow.append(gpow[-1] * g)
    bpx, bpy = bpdiag(x, bx), bpdiag(y, by)
    cp = row_off(m, m + 1)
    G = -(-n // nb)
    mem = {"planes": np.full(max(n, 1) * cp + nb * cp, np.nan),
           "lds": np.full((W, 2, nb, TW), np.nan)}
    wrap0 = max(n, 1) * cp
    np_ = sum(group_positions(gg, n, nb, F, pf) for gg in range(G))
    total = ((np_ - 1) // W) * R + (np_ - 1) % W + R if np_ else 0
    k = np.arange(TW)
    yk = np.array([y[kk] if kk < m else "\0" for kk in k])

    def bp_x(a, b):  # prob(a, b), a <= b
        e = b - a
        return bpx[e * n - e * (e - 1) // 2 + a]

    def describe(q):
        d = dict(on=False, i=0, c0=0, nbg=0, bnd=False, cons=False, stack=[False] * nb,
                 bp_c=[np.float32(0)] * nb, xcj=["\0"] * nb, xci="\0", j_lo=1)
        if not q.valid(n, nb):
            return d
        j_lo, j_hi = q.g * nb + 1, min((q.g + 1) * nb, n)
        d["j_lo"] = j_lo
        d["nbg"] = j_hi - j_lo + 1
        if q.off >= j_hi:
            return d
        i = j_hi - 1 - q.off
        d.update(on=True, i=i, c0=max(0, i + 1 - j_lo), bnd=i + 1 >= j_lo, cons=i >= 1)
        if d["cons"]:
            d["xci"] = x[i - 1]
            for c in range(d["c0"], d["nbg"]):
                jp = j_lo + c
                d["bp_c"][c] = bp_x(i - 1, jp - 1)
                d["xcj"][c] = x[jp - 1]
                d["stack"][c] = d["bp_c"][c] > bound
        return d

    class Wave:
        pass
    waves = []
    for w in range(W):
        v = Wave()
        v.cur = Pos()
        v.cur.advance(w, n, nb, F, pf)
        v.dc = describe(v.cur)
        v.fpos, v.df, v.fs = v.cur.copy(), dict(v.dc), 0
        v.rows = []
        v.s = 0
        v.ksrc = np.zeros(TW)
        v.Am1, v.Am2, v.G2c, v.G3c = ([np.zeros(TW) for _ in range(nb)] for _ in range(4))
        waves.append(v)

    def fetch(v, snap, w, zsnap=None):
        d, s = v.df, v.fs
        kmax = m - s
        ro = row_off(m, s)
        ok = d["on"] and s >= 1
        msk = ok & (k <= kmax)
        r = dict(A=np.zeros(TW), Bw=[np.zeros(TW) for _ in range(nb)], bp=np.zeros(TW, np.float32),
                 yl=np.array(["\0"] * TW))
        if ok:
            kk = k[msk]
            if not d["bnd"]:
                r["A"][msk] = snap["planes"][d["i"] * cp + ro + kk]
            if w == 0:
                src = zsnap if zsnap is not None else snap
                for c in range(d["c0"], d["nbg"]):
                    if c > d["c0"] or not d["bnd"]:
                        r["Bw"][c][msk] = src["planes"][wrap0 + c * cp + ro + kk]
            e2 = s - 1
            ye = e2 * m - e2 * (e2 - 1) // 2
            r["bp"][msk] = bpy[ye + kk]
            r["yl"][msk] = np.array(list(y))[kk + s - 1]
        v.fs += 1
        if v.fs == R:
            v.fs = 0
            v.fpos.advance(W, n, nb, F, pf)
            v.df = describe(v.fpos)
        return r

    def shl1(a):  # lane l <- l + 1 over the TW slots (lane + 64c layout flattened in k order)
        out = np.zeros_like(a)
        out[:-1] = a[1:]
        return out

    snap = {kk: vv.copy() for kk, vv in mem.items()}
    hist = {}  # step -> global snapshot (the staging loads of wave 0's wrap rows)
    for v_i, v in enumerate(waves):  # first rows: PF steps before the wave's first step
        v.rows = [fetch(v, snap, v_i, snap) for _ in range(max(0, pf - v_i))]
    pending = []  # global stores not yet visible: (first visible step, index, values)
    for t in range(total):
        # global stores become visible at the full barriers (before steps t % F == 0)
        keep = []
        for when, idx, val in pending:
            if when <= t:
                mem["planes"][idx] = val
            else:
                keep.append((when, idx, val))
        pending = keep
        snap = {kk: vv.copy() for kk, vv in mem.items()}
        hist[t] = snap
        writes = []
        for w, v in enumerate(waves):
            if not v.cur.valid(n, nb):
                continue
            # wave 0's wrap rows for step t + pf: loaded at step t + pf - zlead
            zs = hist.get(t + pf - zlead, hist[0]) if zlead is not None else snap
            if t < w:
                if t >= w - pf:
                    v.rows.append(fetch(v, snap, w, zs))
                continue
            cr = v.rows.pop(0)
            v.rows.append(fetch(v, snap, w, zs))
            dc = v.dc
            s = v.s
            if dc["on"]:
                kmax = m - s
                msk = k <= kmax
                kk = k[msk]
                i = dc["i"]
                if s == 0:
                    for c in range(dc["c0"], dc["nbg"]):
                        jp = dc["j_lo"] + c
                        v.Am1[c] = np.where(dc["stack"][c] & (k <= m), gpow[jp - 1 - i], 0.0)
                        v.Am2[c], v.G2c[c], v.G3c[c] = np.zeros(TW), np.zeros(TW), np.zeros(TW)
                else:
                    ro = row_off(m, s)
                    A = np.where(msk, gpow[s], 0.0) if dc["bnd"] else cr["A"]
                    for c in range(dc["c0"], dc["nbg"]):
                        if c == dc["c0"] and dc["bnd"]:
                            G1 = np.zeros(TW)
                        elif w == 0:
                            G1 = cr["Bw"][c]
                        else:
                            G1 = snap["lds"][w - 1, (t - 1) & 1, c].copy()
                        G0 = A * g + G1
                        if dc["cons"]:
                            if dc["stack"][c]:
                                G3n, A2 = shl1(v.G3c[c]), shl1(v.Am2[c])
                                g3 = G3n * g
                                src = msk & (cr["bp"] > bound)
                                match = (yk == dc["xci"]) & (cr["yl"] == dc["xcj"][c])
                                a = src & match
                                b = src & ~match
                                bpc = float(dc["bp_c"][c])
                                v.ksrc[a] += A2[a] * stk * bpc * cr["bp"][a].astype(np.float64)
                                g3[a] += A2[a]
                                v.ksrc[b] += A2[b] * stk * sub * bpc * cr["bp"][b].astype(np.float64)
                                g2 = v.G2c[c] * g + g3
                                v.G2c[c] = np.where(msk, g2, v.G2c[c])
                                v.G3c[c] = np.where(msk, g3, v.G3c[c])
                            else:
                                g2 = 0.0
                            Bn = G1 * g + g2
                            if w + 1 < W:
                                writes.append(("lds", (w, t & 1, c, kk), Bn[msk]))
                            else:
                                writes.append(("planes", wrap0 + c * cp + ro + kk, Bn[msk]))
                        if dc["stack"][c]:
                            v.Am2[c], v.Am1[c] = v.Am1[c], A
                        A = G0
                    writes.append(("planes", i * cp + ro + kk, A[msk]))
            v.s += 1
            if v.s == R:
                v.s = 0
                v.cur.advance(W, n, nb, F, pf)
                v.dc = describe(v.cur)
        for name, idx, val in writes:
            if name == "lds":
                mem[name][idx] = val
            else:
                pending.append(((t // F + 1) * F if vis is None else t + vis, idx, val))
    return 1.0 + sum(float(v.ksrc.sum()) for v in waves)


def _case(n, m):
    seqs = ska.random_sequences(2, max(n, m, 1), 0x5EED0C01 + n * 31 + m)
    x, y = seqs[0][:n].lower(), seqs[1][:m].lower()
    # dense base-pair probabilities (every cell a stacking source), so that any
    # value read out of order reaches K
    rng = np.random.default_rng(n * 1000 + m)
    bx = rng.uniform(0.05, 0.6, n * (n - 1) // 2)
    by = rng.uniform(0.05, 0.6, m * (m - 1) // 2)
    return x, bx, y, by


def _ref(x, bx, y, by):
    f = lambda v: float(np.float32(v))  # the CLI's float options, as StemKernel4D rounds them
    return po.stem4d(x, bx, y, by, f(0.8), f(1.0), f(0.5), 0.0)


@pytest.mark.parametrize("n,m,W,F", [(9, 11, 3, 1), (12, 7, 5, 1), (6, 14, 12, 1), (1, 5, 3, 1),
                                     (0, 6, 2, 1), (10, 4, 2, 1), (7, 9, 1, 1), (13, 13, 11, 1),
                                     (12, 17, 4, 8), (10, 21, 12, 8), (16, 13, 4, 8), (5, 30, 12, 8),
                                     (8, 30, 4, 16), (6, 40, 12, 24)])
@pytest.mark.parametrize("pf", [2, 1])
def test_column_schedule_equals_oracle(n, m, W, F, pf):
    x, bx, y, by = _case(n, m)
    assert W <= max(1, m - F - 1)  # the host's limit (the round wrap's lag)
    got = emulate(x, bx, y, by, W, F, pf=pf)
    ref = _ref(x, bx, y, by)
    assert abs(got - ref) <= 1e-12 * abs(ref), (got, ref)


@pytest.mark.parametrize("n,m,W,F", [(9, 11, 3, 1), (12, 7, 5, 1), (13, 13, 11, 1), (1, 5, 3, 1),
                                     (0, 6, 2, 1), (10, 4, 2, 1), (7, 9, 1, 1), (11, 17, 4, 8),
                                     (14, 21, 12, 8), (16, 13, 4, 8), (5, 30, 12, 8), (17, 30, 8, 8)])
@pytest.mark.parametrize("nb", [2, 3, 4])
def test_column_group_schedule_equals_oracle(n, m, W, F, nb):
    """NB columns per group (one chain each per position): groups cut short
    by n (n % NB != 0), the top triangle of a group (positions with fewer
    chains, the first of them a boundary plane), the round wrap of every
    chain."""
    x, bx, y, by = _case(n, m)
    assert W <= max(1, m - F - 1)
    got = emulate(x, bx, y, by, W, F, nb=nb)
    ref = _ref(x, bx, y, by)
    assert abs(got - ref) <= 1e-12 * abs(ref), (got, ref)


def test_emulation_sees_a_broken_schedule():
    """The check has teeth: past the schedule's limit (W > R - 2, the round
    wrap's B' read before it is written) the emulated K is wrong."""
    rng = np.random.default_rng(5)
    x, y = "acguacgua", "ggcaugcaucc"
    bx, by = rng.uniform(0.05, 0.6, 36), rng.uniform(0.05, 0.6, 55)
    ref = _ref(x, bx, y, by)
    for nb in (1, 3):
        assert abs(emulate(x, bx, y, by, 9, nb=nb) - ref) <= 1e-12 * ref
        bad = emulate(x, bx, y, by, 11, nb=nb)
        assert not abs(bad - ref) <= 1e-12 * ref
        # with full barriers every F = 8 steps, W = m - 2 is past the limit m - F - 1
        assert not abs(emulate(x, bx, y, by, 9, F=8, nb=nb) - ref) <= 1e-12 * ref


# the kernel's schedule (stem4d.hip sk_stem4d_col_kernel): rows PF = 1 ahead in
# registers, no full barriers -- a global store is visible V = 2 steps later
# (the writer waits at the end of the next step for a load issued after it,
# then a barrier) -- groups of at least PF + V positions, wave 0's wrap rows
# staged PF + 1 steps ahead, and W <= m - PF - V (host: run_stem4d)
KPF, KV, KNB = 1, 2, 4


def kernel_w_max(m, pf=KPF):
    return max(1, m - pf - KV)


@pytest.mark.parametrize("n,m,W", [(9, 14, 4), (12, 17, 7), (13, 20, 10), (5, 30, 12), (17, 30, 8),
                                   (10, 11, 1), (7, 12, 2), (20, 25, 8)])
@pytest.mark.parametrize("nb,pf", [(4, 1), (3, 1), (4, 2), (1, 4), (2, 4), (3, 4), (2, 3), (3, 2), (2, 2)])
def test_kernel_schedule_equals_oracle(n, m, W, nb, pf):
    """(PF, NB) as the kernel's builds take them (SK4C_PF / SK4C_NB4): the
    limits scale with PF (groups of PF + 2 positions, W <= m - PF - 2)."""
    x, bx, y, by = _case(n, m)
    W = min(W, kernel_w_max(m, pf))
    got = emulate(x, bx, y, by, W, F=KV, nb=nb, pf=pf, vis=KV, zlead=pf + 1)
    ref = _ref(x, bx, y, by)
    assert abs(got - ref) <= 1e-12 * abs(ref), (got, ref)


def test_kernel_schedule_limits_have_teeth():
    """Two waves past the host's W limit (which keeps one wave of margin:
    m - PF - V + 1 is exact here), or a visibility lag longer than the schedule
    allows for, gives a wrong K."""
    x, bx, y, by = _case(17, 20)
    ref = _ref(x, bx, y, by)
    W = kernel_w_max(20)
    assert abs(emulate(x, bx, y, by, W, F=KV, nb=KNB, pf=KPF, vis=KV, zlead=KPF + 1) - ref) <= 1e-12 * ref
    bad = [emulate(x, bx, y, by, W + 2, F=KV, nb=KNB, pf=KPF, vis=KV, zlead=KPF + 1),
           emulate(x, bx, y, by, W, F=KV, nb=KNB, pf=KPF, vis=KV + 2, zlead=KPF + 1)]
    assert all(not abs(b - ref) <= 1e-12 * ref for b in bad), bad


def test_library_col_shape_matches_schedule_limits():
    """The shipped library's column shape (sk_stem4d_col_shape, the bench's
    roofline input) carries the PF this file emulates, and W obeys
    W <= m - PF - 2 for the smallest stacking y of the batch."""
    from stem_kernel_amd.kernel_matrix import stem4d_col_shape
    for lo, hi in [(200, 200), (5, 5), (12, 40), (100, 120), (10, 300)]:
        sh = stem4d_col_shape(lo, hi)
        assert sh["pf"] == KPF
        assert 1 <= sh["waves"] <= kernel_w_max(lo, sh["pf"])
        assert sh["waves"] <= 8
    assert stem4d_col_shape(200, 200)["nb"] == KNB
    assert stem4d_col_shape(10, 300)["nb"] == 1


def _col_cpl(m):
    # the column kernel's class for |y| = m (sk_api.cpp: |y| < 64, 128, 256, 512)
    return next(c for c in (1, 2, 4, 8) if m < 64 * c)


def _phases(m, cpl):
    # stem4d.hip rows(): phase NS runs s .. s_end(NS), s_end = m + 1 - 64 (NS - 1)
    # for NS > 1 and m for NS = 1, from CPL down to 1 (row s holds m - s + 1 cells)
    out, s = [], 1
    for ns in [c for c in (8, 7, 6, 5, 4, 3, 2, 1) if c <= cpl]:
        s_end = m + 1 - 64 * (ns - 1) if ns > 1 else m
        while s <= s_end:
            out.append((s, ns))
            s += 1
    return out


def test_phase_rows_leave_lane_63_of_the_last_slot_empty():
    """Every row 1..m runs in exactly one phase; phase NS's rows hold
    64 (NS-1) .. 64 NS - 1 cells (NS slots suffice, and lane 63 of the last
    slot is never a valid cell, so its lane shift takes nothing from the slot
    past it: wave_shl1_z in stem4d.hip)."""
    for m in range(1, 512):
        cpl = _col_cpl(m)
        rows = _phases(m, cpl)
        assert [s for s, _ in rows] == list(range(1, m + 1)), m
        for s, ns in rows:
            nk = m - s + 1
            assert 1 <= nk <= 64 * ns - 1, (m, s, ns)
            assert ns == 1 or nk >= 64 * (ns - 1), (m, s, ns)
