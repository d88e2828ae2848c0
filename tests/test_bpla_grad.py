"""BPLA gradients: BPLAKernel::compute_gradients
(bpla_kernel/bpla_kernel.cpp:178-401), the per-pair step of bpla_optimizer.

The oracle restates BPLA_Forward / BPLA_Backward / BPLA_ForwardBackword in C
and is pinned by construction plus two properties the reference's algebra
implies: the backward pass's total equals the forward value, and the four
summed terms are the exact derivatives of the forward value (central finite
differences).  The HIP kernel is compared with the oracle within 1e-6
relative (values and each gradient component)."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, mutate_alignment, rel_err


def _alns(seed, n, L, rows=3):
    return [mutate_alignment(s, rows, seed + k) for k, s in enumerate(ska.random_sequences(n, L, seed))]


def _ref(om, kern, pairs):
    p = kern.params
    t = np.array(list(p.score_table))
    vals, grads = [], []
    for a, b in pairs:
        v, d, _ = po.bpla_gradients(om[a], om[b], p.alpha, p.beta, p.gap, p.ext, t)
        vals.append(v)
        grads.append(d)
    return np.array(vals), np.array(grads)


def test_oracle_gradients_are_derivatives():
    _, om = make_examples(_alns(31, 2, 30))
    p = ska.BPLAKernel().params
    t = np.array(list(p.score_table))
    par = [p.alpha, p.beta, p.gap, p.ext]
    v, d, vb = po.bpla_gradients(om[0], om[1], *par, t)
    assert abs(vb / v - 1) < 1e-12  # backward total == forward value
    for k in range(4):
        h = 1e-6 * max(1.0, abs(par[k]))
        up, dn = list(par), list(par)
        up[k] += h
        dn[k] -= h
        fd = (po.bpla_gradients(om[0], om[1], *up, t)[0] -
              po.bpla_gradients(om[0], om[1], *dn, t)[0]) / (2 * h)
        assert abs(fd / d[k] - 1) < 1e-5, (k, fd, d[k])


@pytest.mark.gpu
def test_bpla_gradients_match_oracle(gpu_ctx):
    alns = _alns(41, 4, 45) + _alns(43, 2, 20, rows=1) + [["ACGU-ACGUA", "ACGUAACG-A"]]
    ds, om = make_examples(alns)
    kern = ska.BPLAKernel(alpha=2.0, beta=0.2)
    n = len(alns)
    x, y = (a.astype(np.int32) for a in np.triu_indices(n))
    val, grad = gpu_ctx.bpla_gradients(ds, kern, x, y)
    rv, rg = _ref(om, kern, list(zip(x, y)))
    assert rel_err(val, rv) < 1e-6
    for k in range(4):
        assert rel_err(grad[:, k], rg[:, k]) < 1e-6


@pytest.mark.gpu
def test_bpla_gradients_need_base_pairs(gpu_ctx):
    ds, _ = make_examples(["ACGUACGU", "ACGUAC"], use_bp=False)
    with pytest.raises(ska.StemKernelError):
        gpu_ctx.bpla_gradients(ds, ska.BPLAKernel(), [0], [1])


@pytest.mark.gpu
@pytest.mark.parametrize("normalize", [False, True])
def test_bpla_gradient_gram(gpu_ctx, normalize):
    """CalcMatrix / CalcMatrixN of bpla_optimizer.cpp:52-255 over the GPU
    gradients, against the same formulas over the oracle's."""
    alns = _alns(51, 4, 35)
    ds, om = make_examples(alns)
    kern = ska.BPLAKernel()
    K, G = gpu_ctx.bpla_gradient_gram(ds, kern, normalize=normalize)
    n = len(alns)
    rv, rg = _ref(om, kern, [(i, j) for i in range(n) for j in range(n)])
    RK, RG = rv.reshape(n, n), rg.reshape(n, n, 4).transpose(2, 0, 1)
    RK = np.triu(RK) + np.triu(RK, 1).T  # reference evaluates i <= j only
    RG = np.array([np.triu(g) + np.triu(g, 1).T for g in RG])
    if normalize:
        dk, dg = np.diag(RK).copy(), np.array([np.diag(g) for g in RG])
        sq = np.sqrt(np.outer(dk, dk))
        NK = RK / sq
        NG = np.array([RG[l] / sq - NK / 2 * (dg[l][:, None] / dk[:, None] + dg[l][None, :] / dk[None, :])
                       for l in range(4)])
        np.fill_diagonal(NK, 1.0)
        for l in range(4):
            np.fill_diagonal(NG[l], 0.0)
        RK, RG = NK, NG
    assert rel_err(K, RK) < 1e-6
    for l in range(4):
        assert np.max(np.abs(G[l] - RG[l])) <= 1e-6 * np.max(np.abs(RG[l])) + 1e-12


@pytest.mark.gpu
def test_bpla_gradients_tiny_and_ragged(gpu_ctx):
    """Edge cases of the per-pair tables: one- and two-column alignments
    (the gap / extension derivatives are exactly zero there), and pairs whose
    lengths differ 120-fold, within one batch."""
    alns = [["A"], ["AC", "A-"], ["GGGAAACCC"], [ska.random_sequences(1, 120, 5)[0]],
            ["GGGAAAUCC", "GG-AAAUCC", "GGGAAA-CC"]]
    ds, om = make_examples(alns)
    kern = ska.BPLAKernel()
    n = len(alns)
    x, y = (a.astype(np.int32) for a in np.triu_indices(n))
    val, grad = gpu_ctx.bpla_gradients(ds, kern, x, y)
    rv, rg = _ref(om, kern, list(zip(x, y)))
    assert np.all(np.abs(val / rv - 1) < 1e-6)
    for p in range(x.size):
        floor = 1e-12 * np.max(np.abs(rg[p]))
        assert np.all(np.abs(grad[p] - rg[p]) <= 1e-6 * np.abs(rg[p]) + floor), (x[p], y[p], grad[p], rg[p])


def _c4_set():
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large_bpla.npz"))
    rows = [str(r) for r in g["rows"]]
    alns, k = [], 0
    for nr in g["n_rows"]:
        alns.append(rows[k:k + nr])
        k += nr
    alns = alns[:4]
    ds, om = make_examples(alns)
    n = len(alns)
    x, y = (a.ravel().astype(np.int32) for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
    return ds, om, x, y


@pytest.mark.gpu
def test_bpla_gradients_c4_size_wave_kernel(gpu_ctx):
    """C4's 4-row alignments (L 190-210, dyadic profiles: the wave-per-pair
    kernel with several strips) against the oracle."""
    ds, om, x, y = _c4_set()
    kern = ska.BPLAKernel(alpha=3.0, beta=0.15)
    val, grad = gpu_ctx.bpla_gradients(ds, kern, x, y)
    sel = [0, 1, 6, 11, 15]
    rv, rg = _ref(om, kern, [(int(x[p]), int(y[p])) for p in sel])
    assert rel_err(val[sel], rv) < 1e-6
    for q in range(4):
        assert rel_err(grad[sel, q], rg[:, q]) < 1e-6


@pytest.mark.gpu
@pytest.mark.explib
def test_bpla_gradients_wave_equals_thread_kernel(gpu_ctx, monkeypatch):
    """The wave kernel against the thread-per-pair kernel (experiments build:
    SK_BPLA_GENERAL) on every ordered pair of the C4-size set."""
    ds, om, x, y = _c4_set()
    kern = ska.BPLAKernel(alpha=3.0, beta=0.15)
    val, grad = gpu_ctx.bpla_gradients(ds, kern, x, y)
    monkeypatch.setenv("SK_BPLA_GENERAL", "1")
    gv, gg = gpu_ctx.bpla_gradients(ds, kern, x, y)
    assert rel_err(val, gv) < 1e-9
    for q in range(4):
        assert np.max(np.abs(grad[:, q] - gg[:, q])) <= 1e-9 * np.max(np.abs(gg[:, q]))
