"""Parity at the benchmark configurations' sizes (C2 L=150, NS L=200, C5
L=300, C3 4-D L=200/260, C4 4-row alignments L 190-210), against the oracle
fixtures of tests/golden/make_golden_large.py.

The GPU tests reach every kernel instantiation the benches launch -- DAG stem
register classes MAXK 16, 17, 20, 24, 28 and 32, the profile string kernel's 3-7
strips, 4-D full_dp CPL 4 and 8 and the banded CPL 4 class, BPLA's 4-strip
alignments -- and assert through sk_last_classes that they did.  Tolerance:
1e-6 relative (BASELINE.json north_star, double).

The CPU tests pin the fixtures: the synthetic fold still gives the stored
bpp bytes (SHA-256), the bench's synthetic dataset path builds the same DAG
as the explicit-bpp path the oracle mirrors, and the oracle reproduces a
sample of the stored values bit for bit.
"""
import hashlib
import os

import numpy as np
import pytest

import stem_kernel_amd as ska
from tests.helpers import rel_err

TOL = 1e-6
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DAG = np.load(os.path.join(GOLDEN, "large_dag.npz"))
S4D = np.load(os.path.join(GOLDEN, "large_4d.npz"))
BPLA = np.load(os.path.join(GOLDEN, "large_bpla.npz"))
SETS = ["c2_L150", "ns_L200", "ns15_L200", "ns20_L200", "c5_L300", "wide_L380_420"]
# 6, 7: the log compositions, 7 the north star's LSuStemStrKernel (the CLI's
# --log mode): components as the fixtures' K0 (SuStemKernel()) and K2
# (StringKernel(gap=0.8, alpha=0.2)), which are LSuStemStrKernel()'s
STR_KINDS = {0: ska.SuStemKernel(), 1: ska.SiStemKernel(), 2: ska.StringKernel(gap=0.8, alpha=0.2),
             3: ska.StringKernel(gap=0.8, match=1.0, mismatch=0.8), 4: ska.SuStemStrKernel(),
             5: ska.SiStemStrKernel(), 6: ska.LSuStemKernel(), 7: ska.LSuStemStrKernel()}


def _digest(rows_list):
    h = hashlib.sha256()
    for rows in rows_list:
        for r in rows:
            h.update(np.ascontiguousarray(ska.fold(r.replace("-", "").lower()), np.float64).tobytes())
    return h.hexdigest()


def _expected(name, kind):
    """the fixtures' components, composed in oracle/pyoracle.py kernel_value's
    operation order (def_kernel.h:113-138, :165-190)"""
    p = STR_KINDS[kind].params
    if kind == 6:
        return p.beta * np.log(DAG[f"{name}_K0"]) + 0.0
    if kind == 7:
        return (p.beta * np.log(DAG[f"{name}_K0"]) + 0.0) + (p.alpha * np.log(DAG[f"{name}_K2"]) + 0.0)
    if kind == 4:
        return DAG[f"{name}_K0"] + DAG[f"{name}_K2"]
    if kind == 5:
        return DAG[f"{name}_K1"] + DAG[f"{name}_K3"]
    return DAG[f"{name}_K{kind}"]


def _maxk(nl):
    # sk_api.cpp in_class = dag_stem.hip stem_maxk(nl + 1): 64-node slots per
    # lane for the y's nodes plus one free slot (the sweep's dummy target),
    # rounded up to a multiple of 4 -- except 17 slots (1,024-1,087 nodes), a
    # class of its own
    s = (nl + 1 + 63) // 64
    return 17 if s == 17 else (s + 3) // 4 * 4


def _bpla_alns():
    rows = [str(r) for r in BPLA["rows"]]
    out, k = [], 0
    for nr in BPLA["n_rows"]:
        out.append(rows[k:k + nr])
        k += nr
    return out


# ------------------------------------------------------------------ CPU pins
@pytest.mark.parametrize("name", SETS)
def test_fold_bytes_pinned(name):
    seqs = [str(s) for s in DAG[f"{name}_seqs"]]
    assert _digest([[s] for s in seqs]) == str(DAG[f"{name}_sha"])


def test_fold_bytes_pinned_4d_bpla():
    x = [str(s) for s in S4D["x"]]
    y = [str(s) for s in S4D["y"]]
    assert _digest([[s] for s in x] + [[s] for s in y]) == str(S4D["sha"])
    assert _digest(_bpla_alns()) == str(BPLA["sha"])


def test_synthetic_path_builds_the_oracle_dag():
    """Dataset.synthetic (the bench path: host-threaded fold + build) gives
    the DAG that the explicit-bpp path (sk_dataset_add, mirrored by the
    oracle's MData) gives."""
    seqs = [str(s) for s in DAG["ns_L200_seqs"][:2]] + [str(DAG["wide_L380_420_seqs"][-1])]
    a = ska.Dataset.synthetic(seqs)
    b = ska.Dataset.from_sequences(seqs, bpp=[ska.fold(s.lower()) for s in seqs])
    for i in range(len(seqs)):
        da, db = a.dag(i), b.dag(i)
        for k in da:
            assert np.array_equal(da[k], db[k]), k


def test_wide_set_spans_the_widest_classes():
    seqs = [str(s) for s in DAG["wide_L380_420_seqs"]]
    ds = ska.Dataset.synthetic(seqs)
    ks = {_maxk(int(np.sum(ds.dag(i)["n_edges"] > 0))) for i in range(len(seqs))}
    assert {28, 32} <= ks


def test_oracle_reproduces_sample():
    from oracle import pyoracle as po
    p = ska.SuStemStrKernel().params
    for name in ("ns_L200", "c5_L300"):
        seqs = [str(s) for s in DAG[f"{name}_seqs"]]
        om = [po.OMData([s], [ska.fold(s.lower())], 0.01) for s in seqs[:2]]
        for kind in (0, 3):
            assert po.kernel_value(kind, om[1], om[0], p) == DAG[f"{name}_K{kind}"][1, 0]


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module")
def dag_sets():
    out = {}
    for name in SETS:
        seqs = [str(s) for s in DAG[f"{name}_seqs"]]
        out[name] = ska.Dataset.synthetic(seqs)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
@pytest.mark.parametrize("kind", sorted(STR_KINDS))
def test_dag_pairs_at_config_size(gpu_ctx, dag_sets, name, kind):
    """Every ordered pair (K is asymmetric) of the set, through sk_pairs."""
    ds = dag_sets[name]
    n = len(ds)
    x, y = (a.ravel() for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
    got = gpu_ctx.pairs(ds, STR_KINDS[kind], x, y).reshape(n, n)
    assert rel_err(got, _expected(name, kind)) < TOL
    if kind in (0, 1, 4, 5, 6, 7):
        nl = [int(np.sum(ds.dag(i)["n_edges"] > 0)) for i in range(n)]
        assert gpu_ctx.last_classes()["stem_maxk"] == sorted({_maxk(v) for v in nl})


@pytest.mark.gpu
def test_dag_classes_cover_benched_instantiations(gpu_ctx, dag_sets):
    seen = set()
    for name in SETS:
        ds = dag_sets[name]
        n = len(ds)
        x, y = (a.ravel() for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
        gpu_ctx.pairs(ds, ska.SuStemKernel(), x, y)
        seen |= set(gpu_ctx.last_classes()["stem_maxk"])
    assert {16, 17, 20, 24, 28, 32} <= seen


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ns_L200", "c5_L300"])
def test_gram_normalized_at_config_size(gpu_ctx, dag_sets, name):
    """sk_gram over the set (cells i <= j, mirrored, normalised,
    common/kernel_matrix.cpp:485-575) against the fixture."""
    ds = dag_sets[name]
    raw = _expected(name, 4)
    n = raw.shape[0]
    ref = np.triu(raw) + np.triu(raw, 1).T
    d = np.sqrt(np.diag(raw))
    ref = ref / np.outer(d, d)
    np.fill_diagonal(ref, 1.0)
    got = gpu_ctx.gram(ds, ska.SuStemStrKernel(), normalize=True)
    assert rel_err(got, ref) < TOL
    assert np.array_equal(got, got.T)


@pytest.mark.gpu
def test_stem4d_at_config_size(gpu_ctx):
    xs = [str(s) for s in S4D["x"]]
    ys = [str(s) for s in S4D["y"]]
    band = S4D["band"]
    seqs = sorted(set(xs + ys))
    ds = ska.Dataset.from_sequences(seqs, bpp=[ska.fold(s.lower()) for s in seqs])
    idx = {s: i for i, s in enumerate(seqs)}
    seen = set()
    for k in range(len(xs)):  # one call per pair: a call's class follows its longest y
        got = gpu_ctx.pairs(ds, ska.StemKernel4D(band=int(band[k])), [idx[xs[k]]], [idx[ys[k]]])
        assert rel_err(got, S4D["value"][k:k + 1]) < TOL, k
        cls = gpu_ctx.last_classes()
        seen |= set(cls["stem4d"])
        if int(band[k]) == 0 and len(ys[k]) < 512 and len(xs[k]) <= 2048:
            # the default full_dp kernel is the column-group kernel: it, and
            # only it, ran on this unbanded config-size pair
            cpl = next(c for c in (1, 2, 4, 8) if len(ys[k]) < 64 * c)
            assert cls["stem4d_col"] == [cpl] and cls["stem4d"] == [(cpl, False)], (k, cls)
            seen.add(("col", cpl))
    assert {(4, False), (8, False), (4, True), ("col", 4), ("col", 8)} <= seen


@pytest.mark.gpu
def test_bpla_c4_alignments(gpu_ctx):
    alns = _bpla_alns()
    ds = ska.Dataset.synthetic_alignments(alns)
    n = len(alns)
    x, y = (a.ravel() for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
    for kind, (nobp, sw) in zip((9, 10, 11, 12), [(False, False), (True, False), (False, True),
                                                  (True, True)]):
        got = gpu_ctx.pairs(ds, ska.BPLAKernel(noBP=nobp, SW=sw), x, y).reshape(n, n)
        assert rel_err(got, BPLA[f"K{kind}"]) < TOL, kind
