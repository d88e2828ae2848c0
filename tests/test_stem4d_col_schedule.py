"""CPU check of the column-pipelined 4-D schedule (stem4d.hip
sk_stem4d_col_kernel): a step-by-step numpy emulation of the kernel's waves --
positions, rows, the LDS B' double buffer by step parity, the round-wrap B'
plane, the in-place G0 planes, the PF-rows-ahead fetch cursor -- in which
every read of a step sees memory as it was when the step began and every
write lands when it ends.  A schedule that read anything before it was
written (a race between waves on the GPU) gives a different K; the emulated
K must equal the C oracle's full_dp (stem_kernel/stem_kernel.cpp:282-351)
for several (n, m, W), including W at the host's limit m - 2 and ragged
lengths."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po

PF = 2


def cols(j, F, pf=PF):
    return max(j, F + pf)


class Pos:
    def __init__(self):
        self.j, self.off = 1, 0

    def advance(self, W, n, F, pf=PF):
        self.off += W
        while self.j <= n and self.off >= cols(self.j, F, pf):
            self.off -= cols(self.j, F, pf)
            self.j += 1

    def copy(self):
        q = Pos()
        q.j, q.off = self.j, self.off
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


def emulate(x, bx, y, by, W, F=1, gap=0.8, stack=1.0, subst=0.5, bound=0.0, CPL=None, pf=PF):
    """F: steps between full barriers -- a global store of step u is seen
    from the first multiple of F above u on; LDS stores from the next step."""
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
    mem = {"planes": np.full(max(n, 1) * cp + cp, np.nan), "lds": np.full((W, 2, TW), np.nan)}
    np_ = sum(cols(j, F, pf) for j in range(1, n + 1))
    total = ((np_ - 1) // W) * R + (np_ - 1) % W + R if np_ else 0
    k = np.arange(TW)
    yk = np.array([y[kk] if kk < m else "\0" for kk in k])

    def describe(q):
        on = q.j <= n and q.off < q.j
        d = dict(on=on, i=q.j - 1 - q.off if on else 0, j=q.j if on else 1)
        d["first"] = d["i"] == d["j"] - 1
        d["cons"] = on and d["i"] >= 1
        d["bp_c"] = np.float32(0)
        d["xci"] = d["xcj"] = "\0"
        if d["cons"]:
            e = d["j"] - d["i"]
            d["bp_c"] = bpx[e * n - e * (e - 1) // 2 + d["i"] - 1]
            d["xci"], d["xcj"] = x[d["i"] - 1], x[d["j"] - 1]
        d["stack"] = d["cons"] and d["bp_c"] > bound
        return d

    class Wave:
        pass
    waves = []
    for w in range(W):
        v = Wave()
        v.cur = Pos()
        v.cur.advance(w, n, F, pf)
        v.dc = describe(v.cur)
        v.fpos, v.df, v.fs = v.cur.copy(), dict(v.dc), 0
        v.rows = []
        v.s = 0
        v.ksrc = np.zeros(TW)
        v.Am1, v.Am2, v.G2c, v.G3c = (np.zeros(TW) for _ in range(4))
        waves.append(v)

    def fetch(v, snap, w):
        d, s = v.df, v.fs
        kmax = m - s
        ro = row_off(m, s)
        ok = d["on"] and s >= 1
        msk = ok & (k <= kmax)
        r = dict(A=np.zeros(TW), Bw=np.zeros(TW), bp=np.zeros(TW, np.float32), yl=np.array(["\0"] * TW))
        if ok:
            kk = k[msk]
            if d["first"]:
                r["A"][msk] = gpow[s]
            else:
                r["A"][msk] = snap["planes"][d["i"] * cp + ro + kk]
            if w == 0 and not d["first"]:
                r["Bw"][msk] = snap["planes"][n * cp + ro + kk]
            if d["stack"]:
                e2 = s - 1
                ye = e2 * m - e2 * (e2 - 1) // 2
                r["bp"][msk] = bpy[ye + kk]
                r["yl"][msk] = np.array(list(y))[kk + s - 1]
        v.fs += 1
        if v.fs == R:
            v.fs = 0
            v.fpos.advance(W, n, F, pf)
            v.df = describe(v.fpos)
        return r

    def shl1(a):  # lane l <- l + 1 over the TW slots (lane + 64c layout flattened in k order)
        out = np.zeros_like(a)
        out[:-1] = a[1:]
        return out

    snap = {kk: vv.copy() for kk, vv in mem.items()}
    for v_i, v in enumerate(waves):  # first rows: PF steps before the wave's first step
        v.rows = [fetch(v, snap, v_i) for _ in range(max(0, pf - v_i))]
    pending = []  # global stores not yet visible: (first visible step, index, values)
    for t in range(total):
        # global stores become visible at the full barriers (before steps t % F == 0)
        keep = []
        for vis, idx, val in pending:
            if vis <= t:
                mem["planes"][idx] = val
            else:
                keep.append((vis, idx, val))
        pending = keep
        snap = {kk: vv.copy() for kk, vv in mem.items()}
        writes = []
        for w, v in enumerate(waves):
            if not v.cur.j <= n:
                continue
            if t < w:
                if t >= w - pf:
                    v.rows.append(fetch(v, snap, w))
                continue
            cr = v.rows.pop(0)
            v.rows.append(fetch(v, snap, w))
            dc = v.dc
            s = v.s
            if dc["on"]:
                kmax = m - s
                msk = k <= kmax
                if s == 0:
                    v.Am1 = np.where(dc["stack"] & (k <= m), gpow[dc["j"] - 1 - dc["i"]], 0.0)
                    v.Am2, v.G2c, v.G3c = np.zeros(TW), np.zeros(TW), np.zeros(TW)
                else:
                    ro = row_off(m, s)
                    G3n, A2 = shl1(v.G3c), shl1(v.Am2)
                    if dc["first"]:
                        G1 = np.zeros(TW)
                    elif w == 0:
                        G1 = cr["Bw"]
                    else:
                        G1 = snap["lds"][w - 1, (t - 1) & 1].copy()
                    G0 = cr["A"] * g + G1
                    kk = k[msk]
                    writes.append(("planes", dc["i"] * cp + ro + kk, G0[msk]))
                    if dc["cons"]:
                        g3 = G3n * g
                        if dc["stack"] and s >= 2:
                            src = msk & (cr["bp"] > bound)
                            match = (yk == dc["xci"]) & (cr["yl"] == dc["xcj"])
                            a = src & match
                            b = src & ~match
                            v.ksrc[a] += A2[a] * stk * float(dc["bp_c"]) * cr["bp"][a].astype(np.float64)
                            g3[a] += A2[a]
                            v.ksrc[b] += A2[b] * stk * sub * float(dc["bp_c"]) * cr["bp"][b].astype(np.float64)
                        g2 = v.G2c * g + g3
                        Bn = G1 * g + g2
                        if w + 1 < W:
                            writes.append(("lds", (w, t & 1, kk), Bn[msk]))
                        else:
                            writes.append(("planes", n * cp + ro + kk, Bn[msk]))
                        v.G2c = np.where(msk, g2, v.G2c)
                        v.G3c = np.where(msk, g3, v.G3c)
                    v.Am2, v.Am1 = v.Am1, cr["A"]
            v.s += 1
            if v.s == R:
                v.s = 0
                v.cur.advance(W, n, F, pf)
                v.dc = describe(v.cur)
        for name, idx, val in writes:
            if name == "lds":
                mem[name][idx] = val
            else:
                pending.append(((t // F + 1) * F, idx, val))
    return 1.0 + sum(float(v.ksrc.sum()) for v in waves)


@pytest.mark.parametrize("n,m,W,F", [(9, 11, 3, 1), (12, 7, 5, 1), (6, 14, 12, 1), (1, 5, 3, 1),
                                     (0, 6, 2, 1), (10, 4, 2, 1), (7, 9, 1, 1), (13, 13, 11, 1),
                                     (12, 17, 4, 8), (10, 21, 12, 8), (16, 13, 4, 8), (5, 30, 12, 8),
                                     (8, 30, 4, 16), (6, 40, 12, 24)])
@pytest.mark.parametrize("pf", [2, 1])
def test_column_schedule_equals_oracle(n, m, W, F, pf):
    seqs = ska.random_sequences(2, max(n, m, 1), 0x5EED0C01 + n * 31 + m)
    x, y = seqs[0][:n].lower(), seqs[1][:m].lower()
    # dense base-pair probabilities (every cell a stacking source), so that any
    # value read out of order reaches K
    rng = np.random.default_rng(n * 1000 + m)
    bx = rng.uniform(0.05, 0.6, n * (n - 1) // 2)
    by = rng.uniform(0.05, 0.6, m * (m - 1) // 2)
    assert W <= max(1, m - F - 1)  # the host's limit (the round wrap's lag)
    got = emulate(x, bx, y, by, W, F, pf=pf)
    f = lambda v: float(np.float32(v))  # the CLI's float options, as StemKernel4D rounds them
    ref = po.stem4d(x, bx, y, by, f(0.8), f(1.0), f(0.5), 0.0)
    assert abs(got - ref) <= 1e-12 * abs(ref), (got, ref)


def test_emulation_sees_a_broken_schedule():
    """The check has teeth: past the schedule's limit (W > R - 2, the round
    wrap's B' read before it is written) the emulated K is wrong."""
    rng = np.random.default_rng(5)
    x, y = "acguacgua", "ggcaugcaucc"
    bx, by = rng.uniform(0.05, 0.6, 36), rng.uniform(0.05, 0.6, 55)
    f = lambda v: float(np.float32(v))
    ref = po.stem4d(x, bx, y, by, f(0.8), f(1.0), f(0.5), 0.0)
    assert abs(emulate(x, bx, y, by, 9) - ref) <= 1e-12 * ref
    bad = emulate(x, bx, y, by, 11)
    assert not abs(bad - ref) <= 1e-12 * ref
    # with full barriers every F = 8 steps, W = m - 2 is past the limit m - F - 1
    assert not abs(emulate(x, bx, y, by, 9, F=8) - ref) <= 1e-12 * ref
