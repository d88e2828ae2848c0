"""4-D stem kernel (stem_kernel/): oracle anchors on CPU,
HIP parity (1e-6 relative, double) on the GPU.

Parity anchors: the reference's CLI default without Vienna runs
NormalBasePair with bp_bound 1.0, which makes every kernel value 1
(SURVEY.md §8c probe anchor); the -p path (bp_model 0) uses the dataset's
base-pairing probabilities.  Sequences are lowercased as the reference loader
does (common/example.cpp:29-36)."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, rel_err

TOL = 1e-6


def _seqs():
    s = ska.random_sequences(4, 30, 0x5EED0003) + ska.random_sequences(2, 70, 0x5EED0013)
    s += ska.random_sequences(1, 64, 3) + ska.random_sequences(1, 63, 4)
    s += ["GGGGAAAACCCC", "A", "ACGUN"]
    return s


def _oracle(seqs, kern, pairs):
    p = kern.params
    out = []
    for a, b in pairs:
        xa, xb = seqs[a], seqs[b]
        out.append(po.stem4d(xa.lower(), ska.fold(xa), xb.lower(), ska.fold(xb), p.gap, p.stack,
                             p.subst, p.bp_bound, p.bp_model, p.loop, p.len_band))
    return np.array(out)


def test_oracle_normal_basepair_is_one():
    s = [q.lower() for q in ska.random_sequences(3, 25, 11)]
    for a in s:
        for b in s:
            assert po.stem4d(a, None, b, None, bp_bound=1.0, model=1) == 1.0
            assert po.stem4d(a, None, b, None, bp_bound=1.0, model=2) == 1.0


def test_oracle_empty_and_defaults():
    assert po.stem4d("", None, "acgu", np.zeros(6)) == 1.0
    p = ska.StemKernel4D().params
    assert p.kind == 13 and p.gap == float(np.float32(0.8)) and p.stack == 1.0
    assert p.subst == 0.5 and p.bp_bound == 0.0 and p.len_band == 0


@pytest.mark.gpu
@pytest.mark.parametrize("model,bound", [(0, 0.0), (0, 0.3), (1, 0.5), (2, 0.5), (1, 1.0)])
def test_stem4d_gram_matches_oracle(gpu_ctx, model, bound):
    seqs = _seqs()
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(bp_model=model, bp_bound=bound)
    got = gpu_ctx.gram(ds, kern)
    n = len(seqs)
    iu = list(zip(*np.triu_indices(n)))
    ref = _oracle(seqs, kern, iu)
    assert rel_err(got[tuple(np.array(iu).T)], ref) < TOL
    if model == 1 and bound == 1.0:
        assert np.all(got == 1.0)


@pytest.mark.gpu
def test_stem4d_params_and_predict(gpu_ctx):
    seqs = ska.random_sequences(5, 40, 0x5EED0033)
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(gap=0.5, stack=1.5, subst=0.25, loop=4)
    x = np.array([0, 1, 4, 2], np.int32)
    y = np.array([3, 1, 0, 4], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    ref = _oracle(seqs, kern, list(zip(x, y)))
    assert rel_err(got, ref) < TOL
    row = gpu_ctx.test_row(ds, 1, ds, kern)
    ref = _oracle(seqs, kern, [(i, 1) for i in range(5)])
    assert rel_err(row, ref) < TOL


def test_oracle_band_wide_equals_full_dp():
    """partial_dp with a band wider than both sequences computes every cell."""
    s = ska.random_sequences(3, 24, 21) + ska.random_sequences(1, 17, 22)
    for a in range(4):
        for b in range(4):
            x, y = s[a], s[b]
            full = po.stem4d(x.lower(), ska.fold(x), y.lower(), ska.fold(y))
            wide = po.stem4d(x.lower(), ska.fold(x), y.lower(), ska.fold(y), band=64)
            assert wide == full


@pytest.mark.gpu
@pytest.mark.parametrize("band", [1, 3, 8, 100])
def test_stem4d_banded_matches_oracle(gpu_ctx, band):
    """partial_dp (-b): band constraints and the boundary approximations."""
    seqs = ska.random_sequences(3, 40, 0x5EED0043) + ska.random_sequences(2, 27, 9)
    seqs += ska.random_sequences(1, 70, 10) + ["GGGAAACCC", "A"]
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(band=band)
    n = len(seqs)
    iu = list(zip(*np.triu_indices(n)))
    got = gpu_ctx.gram(ds, kern)
    ref = _oracle(seqs, kern, iu)
    assert rel_err(got[tuple(np.array(iu).T)], ref) < TOL
    # asymmetric lengths in both orders
    x = np.array([3, 0, 5, 6], np.int32)
    y = np.array([0, 3, 1, 2], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    assert rel_err(got, _oracle(seqs, kern, list(zip(x, y)))) < TOL


@pytest.mark.gpu
def test_stem4d_rejects_alignments(gpu_ctx):
    ds, _ = make_examples([["ACGUACGU", "ACG-ACGU"], "ACGUAC"])
    with pytest.raises(ska.StemKernelError):
        gpu_ctx.gram(ds, ska.StemKernel4D())
