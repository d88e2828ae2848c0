"""The synthetic Nussinov-Boltzmann fold (csrc/host/synth.cpp fold_nussinov,
the benches' stand-in for pf_fold) against a scalar restatement of its loops
in plain Python floats (IEEE double, no contraction): the diagonal-order,
four-cells-side-by-side, AVX2-cloned build must give the same bits as the
scalar inside/outside recursion, with and without GU pairs."""
import math

import numpy as np
import pytest

import stem_kernel_amd as ska


def _scalar_fold(seq, no_gu):
    n = len(seq)
    s, hp = 2.0, 3
    inv_s = 1.0 / s
    inv_s2 = inv_s * inv_s

    def w(a, b):
        a, b = a.lower().replace("t", "u"), b.lower().replace("t", "u")
        if (a, b) in (("g", "c"), ("c", "g")):
            return math.exp(1.5)
        if (a, b) in (("a", "u"), ("u", "a")):
            return math.exp(1.0)
        if not no_gu and (a, b) in (("g", "u"), ("u", "g")):
            return math.exp(0.5)
        return 0.0
    # X(i, i + e) for e = -1 .. n-1
    Q = {(i, -1): 1.0 for i in range(n + 1)}
    B, O, P = {}, {}, {}
    for e in range(hp + 1, n):
        for i in range(n - e):
            B[(i, e)] = w(seq[i], seq[i + e]) * inv_s2
    g = lambda X, i, e: X.get((i, e), 0.0)
    for d in range(n):
        for i in range(n - d):
            v = g(Q, i, d - 1) * inv_s
            for t in range(d - hp):
                v += g(Q, i, t - 1) * g(B, i + t, d - t) * g(Q, i + t + 1, d - t - 2)
            Q[(i, d)] = v
    Z = Q[(0, n - 1)]
    O[(0, n - 1)] = 1.0
    for d in range(n - 1, -1, -1):
        for i in range(n - d):
            o = g(O, i, d)
            if o == 0.0:
                continue
            if d >= 1:
                O[(i, d - 1)] = g(O, i, d - 1) + o * inv_s
            for t in range(d - hp):
                b = g(B, i + t, d - t)
                left = g(Q, i, t - 1)
                inner = g(Q, i + t + 1, d - t - 2)
                if t >= 1:
                    O[(i, t - 1)] = g(O, i, t - 1) + o * b * inner
                O[(i + t + 1, d - t - 2)] = g(O, i + t + 1, d - t - 2) + o * b * left
                P[(i + t, d - t)] = g(P, i + t, d - t) + o * left * b * inner
    return np.array([g(P, i, j - i) / Z for i in range(n) for j in range(i + 1, n)])


@pytest.mark.parametrize("n,seed", [(9, 1), (17, 2), (30, 3), (41, 4)])
@pytest.mark.parametrize("no_gu", [False, True])
def test_fold_nussinov_bit_identical_to_scalar(n, seed, no_gu):
    seq = ska.random_sequences(1, n, 0x5EED5000 + seed)[0]
    got = ska.fold(seq, no_gu=no_gu)
    ref = _scalar_fold(seq, no_gu)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)
