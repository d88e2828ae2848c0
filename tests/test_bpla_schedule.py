"""CPU check of the BPLA kernel's systolic schedule (bpla.hip), emulated in
numpy lane by lane: DPP wave_shr for the row above, last step's received
values as the diagonal, the per-wave LDS boundary row between 64-row strips.
The score of each cell is the product's (float products as the reference
writes them, bpla_kernel.cpp:24-62); the DP must equal the oracle's
local_alignment_exp / _max (bpla_kernel.cpp:64-157)."""
import math

import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, mutate_alignment

TB = None


def _score_matrix(ds, ix, iy, params, bp):
    px, _ = ds.profile(ix)
    py, _ = ds.profile(iy)
    tb = np.array(list(params.score_table)).reshape(4, 4)
    wx = ds.bpla_weights(ix)
    wy = ds.bpla_weights(iy)
    Lx, Ly = px.shape[0], py.shape[0]
    S = np.zeros((Lx, Ly))
    for i in range(Lx):
        for j in range(Ly):
            v, n = 0.0, np.float32(0)
            for k in range(4):
                if px[i, k] == 0:
                    continue
                for l in range(4):
                    if py[j, l] == 0:
                        continue
                    n = np.float32(n + np.float32(px[i, k] * py[j, l]))
                    v += tb[k, l] * float(px[i, k]) * float(py[j, l])
            la = 0.0 if n == 0 else v / float(n)
            if bp:
                pp = np.float32(np.float32(wx[1][i] * wy[1][j]) + np.float32(wx[0][i] * wy[0][j]))
                uu = np.float32(wx[2][i] * wy[2][j])
                la = params.alpha * float(pp) + float(uu) * la
            S[i, j] = la
    return S


def _systolic(S, beta, gap, ext, sw):
    """The kernel's lane/step schedule; lanes are a numpy axis."""
    Lx, Ly = S.shape
    if Lx == 0 or Ly == 0:
        return 0.0 if sw else 1.0
    bg, be = math.exp(beta * gap), math.exp(beta * ext)
    lane = np.arange(64)
    B = np.zeros((4, Ly + 2))  # boundary rows M, X, Y, X2
    result, mmax = None, 0.0
    for strip in range((Lx + 63) // 64):
        i = strip * 64 + lane + 1
        ok = i <= Lx
        l = np.zeros((5, 64))  # lM lX lY lX2 lY2
        d = np.zeros((3, 64))  # dM dX dY
        for t in range(Ly + 64):
            j = t - lane + 1
            b0 = B[:, t + 1] if t + 1 <= Ly else np.zeros(4)
            up = np.empty((4, 64))
            up[:, 1:] = l[:4, :-1]  # wave_shr: lane k gets lane k-1
            up[:, 0] = b0
            act = (j >= 1) & (j <= Ly)
            for k in np.nonzero(act)[0]:
                s = S[i[k] - 1, j[k] - 1] if ok[k] else 0.0
                upM, upX, upY, upX2 = up[:, k]
                lM, lX, lY, lX2, lY2 = l[:, k]
                dM, dX, dY = d[:, k]
                if not sw:
                    nM = math.exp(beta * s) * (1.0 + dX + dY + dM)
                    nX = bg * upM + be * upX
                    nY = bg * (lM + lX) + be * lY
                    nX2 = upM + upX2
                    nY2 = lM + lX2 + lY2
                else:
                    nM = max(max(max(0.0, dM), dX), dY) + s
                    nX = max(upM + gap, upX + ext)
                    nY = max(max(lM + gap, lX + gap), lY + ext)
                    nX2 = nY2 = 0.0
                if ok[k]:
                    l[:, k] = (nM, nX, nY, nX2, nY2)
                    mmax = max(mmax, nM)
                    if i[k] == Lx and j[k] == Ly:
                        result = 1.0 + nX2 + nY2 + nM
                if k == 63:
                    B[:, j[k]] = (nM, nX, nY, nX2)
            d = up[:3].copy()
    return mmax if sw else result


@pytest.mark.parametrize("kind", [9, 10, 11, 12])
def test_systolic_schedule_matches_oracle(kind):
    seqs = ska.random_sequences(3, 70, 0x5EED0003)
    seqs += [seqs[0][:5], seqs[1][:64] + seqs[2][:1]]
    alns = [mutate_alignment(seqs[0], 3, 11)]
    ds, om = make_examples(seqs + alns)
    p = ska.BPLAKernel(noBP=kind in (10, 12), SW=kind in (11, 12)).params
    for ix, iy in [(0, 1), (3, 2), (4, 0), (5, 1), (2, 4)]:
        S = _score_matrix(ds, ix, iy, p, bp=kind in (9, 11))
        got = _systolic(S, p.beta, p.gap, p.ext, sw=kind in (11, 12))
        ref = po.kernel_value(kind, om[ix], om[iy], p)
        assert abs(got - ref) <= 1e-12 * abs(ref), (ix, iy, got, ref)
