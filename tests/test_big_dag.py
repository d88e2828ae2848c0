"""Y examples beyond the DAG stem kernel's register classes: more than 2,048
non-leaf nodes (L = 500) or a stem edge gap over 1,023 (caller bpp, L =
1,100) go to sk_dag_stem_big_kernel (dag_stem_big.hip).  The reference has no
size limit (stem_kernel_lite/stem_kernel.cpp:14-95).

Fixtures: tests/golden/make_golden_big.py (CPU oracle).  The big-y kernel is
also forced onto register-class sizes (diagnostic SK_FORCE_BIG_Y=1) and
checked against the large-config fixtures.  Tolerance 1e-6 relative.
"""
import hashlib
import os

import numpy as np
import pytest

import stem_kernel_amd as ska
from tests.helpers import rel_err

TOL = 1e-6
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BIG = np.load(os.path.join(GOLDEN, "big_dag.npz"))
KINDS = {0: ska.SuStemKernel(), 1: ska.SiStemKernel(), 4: ska.SuStemStrKernel(),
         5: ska.SiStemStrKernel()}


def _expected(kind):
    return {0: BIG["K0"], 1: BIG["K1"], 4: BIG["K0"] + BIG["K2"], 5: BIG["K1"] + BIG["K3"]}[kind]


def _seqs():
    return [str(s) for s in BIG["seqs"]]


def test_fold_bytes_pinned():
    h = hashlib.sha256()
    for s in _seqs():
        h.update(np.ascontiguousarray(ska.fold(s.lower()), np.float64).tobytes())
    assert h.hexdigest() == str(BIG["sha"])


def test_fixture_sizes_exceed_register_classes():
    ds = ska.Dataset.synthetic(_seqs())
    nl = [int(np.sum(ds.dag(i)["n_edges"] > 0)) for i in range(len(ds))]
    assert nl[0] > 2048 and nl[1] > 2048 and nl[2] <= 2048
    g = ska.Dataset.from_sequences([str(BIG["gap_seq"])], bpp=[BIG["gap_bpp"]]).dag(0)
    assert int(g["edge_gaps"].max()) > 1023


@pytest.fixture(scope="module")
def big_set():
    return ska.Dataset.synthetic(_seqs())


@pytest.mark.gpu
@pytest.mark.parametrize("kind", sorted(KINDS))
def test_big_y_pairs(gpu_ctx, big_set, kind):
    n = len(big_set)
    x, y = (a.ravel() for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
    got = gpu_ctx.pairs(big_set, KINDS[kind], x, y).reshape(n, n)
    assert rel_err(got, _expected(kind)) < TOL
    classes = gpu_ctx.last_classes()["stem_maxk"]
    assert 0 in classes and any(k > 0 for k in classes), classes  # both kernels ran


@pytest.mark.gpu
def test_big_y_gram_normalized(gpu_ctx, big_set):
    raw = _expected(4)
    ref = np.triu(raw) + np.triu(raw, 1).T
    d = np.sqrt(np.diag(raw))
    ref = ref / np.outer(d, d)
    np.fill_diagonal(ref, 1.0)
    got = gpu_ctx.gram(big_set, ska.SuStemStrKernel(), normalize=True)
    assert rel_err(got, ref) < TOL


@pytest.mark.gpu
def test_long_gap_edge(gpu_ctx, big_set):
    seqs = _seqs()
    ds = ska.Dataset.from_sequences([seqs[0], seqs[2], str(BIG["gap_seq"])],
                                    bpp=[ska.fold(seqs[0].lower()), ska.fold(seqs[2].lower()),
                                         BIG["gap_bpp"]])
    for kind in (0, 1):
        got = gpu_ctx.pairs(ds, KINDS[kind], [2, 0, 2], [2, 2, 1])
        assert rel_err(got, BIG[f"gap_K{kind}"]) < TOL, kind
        assert 0 in gpu_ctx.last_classes()["stem_maxk"]


@pytest.mark.gpu
@pytest.mark.explib
@pytest.mark.parametrize("name", ["ns_L200", "wide_L380_420"])
def test_forced_big_kernel_at_register_sizes(gpu_ctx, monkeypatch, name):
    dag = np.load(os.path.join(GOLDEN, "large_dag.npz"))
    ds = ska.Dataset.synthetic([str(s) for s in dag[f"{name}_seqs"]])
    n = len(ds)
    x, y = (a.ravel() for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
    monkeypatch.setenv("SK_FORCE_BIG_Y", "1")
    for kind in (0, 1):
        got = gpu_ctx.pairs(ds, KINDS[kind], x, y).reshape(n, n)
        assert rel_err(got, dag[f"{name}_K{kind}"]) < TOL, kind
        assert gpu_ctx.last_classes()["stem_maxk"] == [0]
