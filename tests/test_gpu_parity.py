"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Tolerance: 1e-6 relative (BASELINE.json north_star, double precision); the
observed error is ~1e-14 (the GPU sums the same positive terms in another
order).
"""
import math

import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, mutate_alignment, rel_err

TOL = 1e-6
pytestmark = pytest.mark.gpu

KERNELS = [
    ska.SuStemKernel(), ska.SiStemKernel(), ska.StringKernel(gap=0.8, alpha=0.2),
    ska.StringKernel(gap=0.8, match=1.0, mismatch=0.8), ska.SuStemStrKernel(),
    ska.SiStemStrKernel(), ska.LSuStemKernel(), ska.LSuStemStrKernel(),
]


def oracle_matrix(om, kern, rows=None, cols=None):
    rows = range(len(om)) if rows is None else rows
    cols = range(len(om)) if cols is None else cols
    return np.array([[po.kernel_value(kern.params.kind, om[i], om[j], kern.params) for j in cols]
                     for i in rows])


@pytest.fixture(scope="module")
def small_set():
    seqs = ska.random_sequences(6, 60, 0x5EED0001) + ska.random_sequences(2, 45, 99)
    return make_examples(seqs)


@pytest.mark.parametrize("kern", KERNELS, ids=lambda k: type(k).__name__ + str(k.params.kind))
def test_gram_all_kinds(gpu_ctx, small_set, kern):
    ds, om = small_set
    n = len(om)
    got = gpu_ctx.gram(ds, kern)
    ref = oracle_matrix(om, kern)
    # the reference evaluates K(i,j) for i<=j and mirrors (kernel_matrix.cpp:44-55)
    up = np.triu_indices(n)
    assert rel_err(got[up], ref[up]) < TOL
    assert np.array_equal(got, got.T)


def test_gram_normalize(gpu_ctx, small_set):
    ds, om = small_set
    kern = ska.SuStemStrKernel()
    got = gpu_ctx.gram(ds, kern, normalize=True)
    raw = oracle_matrix(om, kern)
    n = len(om)
    ref = raw.copy()
    for i in range(n - 1):
        for j in range(i + 1, n):
            ref[i, j] = raw[i, j] / math.sqrt(raw[i, i] * raw[j, j])
            ref[j, i] = ref[i, j]
    np.fill_diagonal(ref, 1.0)
    assert rel_err(got, ref) < TOL
    assert np.all(np.diag(got) == 1.0)


def test_asymmetric_pairs(gpu_ctx, small_set):
    """K(a,b) != K(b,a) for the DAG kernel; both orders match the oracle."""
    ds, om = small_set
    kern = ska.SuStemKernel()
    x = np.array([0, 1, 2, 3, 5], np.int32)
    y = np.array([1, 0, 4, 2, 3], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    ref = np.array([po.su_stem(om[a], om[b]) for a, b in zip(x, y)])
    assert rel_err(got, ref) < TOL
    assert abs(got[0] / got[1] - 1) > 1e-6


@pytest.mark.parametrize("band", [0, 3, 10])
@pytest.mark.parametrize("th", [0.01, 0.05])
def test_stem_params(gpu_ctx, band, th):
    seqs = ska.random_sequences(5, 70, 1234 + band)
    ds, om = make_examples(seqs, th=th)
    kern = ska.SuStemKernel(loop_gap=0.35, beta=0.5, len_band=band)
    got = gpu_ctx.gram(ds, kern)
    ref = np.array([[po.su_stem(om[i], om[j], 0.35, 0.5, band) for j in range(5)] for i in range(5)])
    up = np.triu_indices(5)
    assert rel_err(got[up], ref[up]) < TOL


def test_alignments_and_iupac(gpu_ctx):
    base = ska.random_sequences(3, 55, 77)
    alns = [mutate_alignment(base[0], 3, 1), mutate_alignment(base[1], 2, 2), [base[2]],
            ["ACGUNRYKMSWACGUACGGGAAACCCUUUGGGAAACCCRY" + "acgu" * 3]]
    ds, om = make_examples(alns)
    for kern in (ska.SuStemStrKernel(), ska.SiStemStrKernel()):
        got = gpu_ctx.gram(ds, kern)
        ref = oracle_matrix(om, kern)
        up = np.triu_indices(len(alns))
        assert rel_err(got[up], ref[up]) < TOL


def test_edge_cases(gpu_ctx):
    """Empty DAGs (nothing above the threshold), very short and ragged inputs."""
    seqs = ["ACGU", "AAAAAAAAAAAA", ska.random_sequences(1, 33, 5)[0], "GGGGAAACCCC",
            ska.random_sequences(1, 90, 6)[0]]
    ds, om = make_examples(seqs)
    for kern in (ska.SuStemKernel(), ska.StringKernel(), ska.SuStemStrKernel()):
        got = gpu_ctx.gram(ds, kern)
        ref = oracle_matrix(om, kern)
        up = np.triu_indices(len(seqs))
        assert rel_err(got[up], ref[up]) < TOL
    # no bp information at all: MData(ma) -> stem 0, string unweighted
    ds2, om2 = make_examples(seqs[:3], use_bp=False)
    got = gpu_ctx.gram(ds2, ska.StringKernel())
    ref = oracle_matrix(om2, ska.StringKernel())
    up = np.triu_indices(3)
    assert rel_err(got[up], ref[up]) < TOL


def test_predict_paths(gpu_ctx, small_set):
    ds, om = small_set
    test_seqs = ska.random_sequences(3, 58, 4242)
    dt, omt = make_examples(test_seqs)
    kern = ska.SuStemStrKernel()
    n = len(om)
    # test row with sv subset: out[x] = K(train[x], test[t])
    sv = [1, 4, 6]
    row, slf = gpu_ctx.test_row(dt, 1, ds, kern, sv_index=sv, self_value=True)
    for x in range(n):
        if x in sv:
            ref = po.kernel_value(kern.params.kind, om[x], omt[1], kern.params)
            assert abs(row[x] / ref - 1) < TOL
        else:
            assert row[x] == 0.0
    assert abs(slf / po.kernel_value(kern.params.kind, omt[1], omt[1], kern.params) - 1) < TOL
    diag = gpu_ctx.diagonal(ds, kern)
    ref = [po.kernel_value(kern.params.kind, om[i], om[i], kern.params) for i in range(n)]
    assert rel_err(diag, ref) < TOL
    m, self_ = gpu_ctx.test_matrix(dt, ds, kern, norm_test=True, normalize=True)
    raw = np.array([[po.kernel_value(kern.params.kind, om[j], omt[i], kern.params) for j in range(n)]
                    for i in range(3)])
    sref = np.array([po.kernel_value(kern.params.kind, omt[i], omt[i], kern.params) for i in range(3)])
    ref = raw / np.sqrt(np.outer(sref, np.array(ref)))
    assert rel_err(m, ref) < TOL
    assert rel_err(self_, sref) < TOL


def test_libsvm_output(gpu_ctx, small_set):
    ds, om = small_set
    km = ska.KernelMatrix(gpu_ctx)
    km.calculate(ds, ska.SuStemKernel())
    import io
    buf = io.StringIO()
    km.print(buf)
    lines = buf.getvalue().splitlines()
    assert len(lines) == len(om)
    first = lines[0].split()
    assert first[0] == "+1" and first[1] == "1" or first[1] == "0:1"
    assert first[1] == "0:1"
    assert float(first[2].split(":")[1]) == pytest.approx(km.matrix[0, 0], rel=1e-5)


@pytest.mark.gpu
def test_row_traffic_counts(gpu_ctx):
    """sk_dataset_row_traffic (the DAG roofline's compulsory bytes, bench.py
    dag_row_bytes): per example, stored rows <= rows, counts >= 0,
    y_slots = the non-leaf node count."""
    seqs = ska.random_sequences(6, 120, 0x5EED0707)
    ds = ska.Dataset.synthetic(seqs)
    gpu_ctx.upload(ds)
    for i in range(len(seqs)):
        t = ds.row_traffic(i)
        assert 0 <= t["stored"] <= t["rows"]
        assert min(t.values()) >= 0
        assert t["y_slots"] == int(np.sum(ds.dag(i)["n_edges"] > 0))
