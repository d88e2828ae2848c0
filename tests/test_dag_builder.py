"""Host preprocessing parity: the product's MData/DAG builder
(stem_kernel_amd/csrc/host/example_build.cpp) against the oracle's
restatement of stem_kernel_lite/data.cpp -- node order, edges, gaps, weights,
bp frequencies, roots, max parents and position weights, all bit-exact."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import mutate_alignment


def check_same(rows, th, use_bp=True):
    bpps = [ska.fold(r.replace("-", "").lower()) for r in rows] if use_bp else None
    ds = ska.Dataset()
    ds.add("+1", rows, bpps, th=th, use_bp=use_bp)
    p = ds.dag(0)
    o = po.OMData(rows, bpps, th, use_bp).dag()
    for k in o:
        assert np.array_equal(p[k], o[k]), (k, p[k][:8], o[k][:8])
    return p


@pytest.mark.parametrize("L", [1, 2, 5, 12, 40, 80, 150])
@pytest.mark.parametrize("th", [0.01, 0.05, 0.3])
def test_single_sequences(L, th):
    for s in ska.random_sequences(2, L, 100 + L):
        check_same([s], th)


def test_L200_shape_matches_survey_probe():
    # |V|~1143, |E|~2994 at L=200, th=0.01 (same synthetic model)
    shapes = [check_same([s], 0.01)["first"].size for s in ska.random_sequences(3, 200, 9)]
    assert 900 < np.mean(shapes) < 1400


@pytest.mark.parametrize("seed", range(5))
def test_alignments(seed):
    base = ska.random_sequences(1, 70, 500 + seed)[0]
    rows = mutate_alignment(base, 2 + seed % 3, seed)
    check_same(rows, 0.01)


def test_iupac_gaps_and_case():
    check_same(["acgunRYKM-SWBDHVNacgGGGAAACCCuuuGGGAAAACCC"], 0.01)
    check_same(["GGGGAAACCCCUUUU", "GG-GAAACCC-UUUU"], 0.02)


def test_no_pairs_and_no_bp():
    p = check_same(["AAAAAAAAAAAA"], 0.01)
    assert p["first"].size == 0 and p["roots"].size == 0
    check_same(["ACGUACGU"], 0.01, use_bp=False)


def test_fold_is_probability():
    for s in ska.random_sequences(3, 90, 3):
        b = ska.fold(s)
        n = len(s)
        M = np.zeros((n, n))
        M[np.triu_indices(n, 1)] = b
        M = M + M.T
        assert np.all(b >= 0) and np.all(M.sum(axis=1) <= 1 + 1e-12)


def test_synthetic_alignments_match_per_example_build():
    """sk_dataset_add_synthetic_rows (threaded) == sk_dataset_add per example."""
    from tests.helpers import make_examples, mutate_alignment
    base = ska.random_sequences(3, 60, 9)
    alns = [mutate_alignment(b, 3, i) for i, b in enumerate(base)]
    ds = ska.Dataset.synthetic_alignments(alns, threads=3)
    ds2, _ = make_examples(alns)
    for i in range(3):
        a, b = ds.dag(i), ds2.dag(i)
        assert all(np.array_equal(a[k], b[k]) for k in a)
        for u, v in zip(ds.bpla_weights(i), ds2.bpla_weights(i)):
            assert np.array_equal(u, v)
