"""Golden vectors (tests/golden/lite_small.npz, made by make_golden.py).

CPU: the oracle reproduces the stored values bit-exactly and the product DAG
builder reproduces the stored DAG shapes.  GPU: the engine matches the stored
values within 1e-6 relative."""
import os

import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "lite_small.npz"))


def examples():
    rows, ex_rows = list(G["rows"]), list(G["ex_rows"])
    offs = np.concatenate([[0], np.cumsum(G["bpp_len"])])
    bpps = [G["bpp"][offs[i]:offs[i + 1]] for i in range(len(rows))]
    out, k = [], 0
    for nr in ex_rows:
        out.append((rows[k:k + nr], bpps[k:k + nr]))
        k += nr
    return out


def test_oracle_reproduces_golden():
    ex = examples()
    om = [po.OMData(r, b, 0.01) for r, b in ex]
    p = ska.SuStemStrKernel().params
    for kind in range(8):
        ref = G[f"K{kind}"]
        for i in range(len(om)):
            for j in range(len(om)):
                assert po.kernel_value(kind, om[i], om[j], p) == ref[i, j]
    nv = [str(s) for s in G["naive_seqs"]]
    assert all(po.naive_string(a, b, 0.8) == G["naive"][i, j]
               for i, a in enumerate(nv) for j, b in enumerate(nv))


def test_product_dag_shapes_golden():
    ds = ska.Dataset()
    for r, b in examples():
        ds.add("+1", r, b, th=0.01)
    got = np.array([[ds.shape(i)[k] for k in (0, 1, 2, 3)] for i in range(len(ds))])
    assert np.array_equal(got, G["shapes"])


@pytest.mark.gpu
def test_gpu_matches_golden(gpu_ctx):
    ds = ska.Dataset()
    for r, b in examples():
        ds.add("+1", r, b, th=0.01)
    n = len(ds)
    x, y = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    for kind, kern in enumerate([ska.SuStemKernel(), ska.SiStemKernel(), ska.StringKernel(),
                                 ska.StringKernel(match=1.0, mismatch=0.8), ska.SuStemStrKernel(),
                                 ska.SiStemStrKernel(), ska.LSuStemKernel(), ska.LSuStemStrKernel()]):
        assert kern.params.kind == kind
        got = gpu_ctx.pairs(ds, kern, x.ravel(), y.ravel()).reshape(n, n)
        ref = G[f"K{kind}"]
        assert np.max(np.abs(got - ref) / np.abs(ref)) < 1e-6, kind
    nv = [str(s) for s in G["naive_seqs"]]
    dn = ska.Dataset()
    for s in nv:
        dn.add("+1", [s], use_bp=False)
    m = len(nv)
    x, y = np.meshgrid(np.arange(m), np.arange(m), indexing="ij")
    got = gpu_ctx.pairs(dn, ska.NaiveStringKernel(0.8), x.ravel(), y.ravel()).reshape(m, m)
    assert np.max(np.abs(got - G["naive"]) / np.abs(G["naive"])) < 1e-6
