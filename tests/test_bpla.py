"""BPLA kernel (bpla_kernel/): host weights (CPU, bit-exact)
and HIP parity against the oracle (GPU, 1e-6 relative; max-plus SW modes
only reorder nothing, so they agree to rounding of the score)."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, mutate_alignment, rel_err

TOL = 1e-6
MODES = [(False, False), (True, False), (False, True), (True, True)]


def _examples():
    seqs = ska.random_sequences(5, 90, 0x5EED0003) + ska.random_sequences(2, 64, 7)
    seqs += ["GGGAAACCC", "A", "ACGUN"]  # short, length 1, IUPAC N
    base = ska.random_sequences(2, 70, 0x5EED0013)
    alns = [mutate_alignment(base[0], 4, 3), mutate_alignment(base[1], 3, 4)]
    alns.append(["ACGU-GRYAC", "AC-UUGCYAC"])  # IUPAC codes with gaps
    return seqs + alns


@pytest.fixture(scope="module")
def bpla_set():
    return make_examples(_examples())


def test_bpla_weights_match_oracle(bpla_set):
    ds, om = bpla_set
    for i in range(len(om)):
        got = ds.bpla_weights(i)
        ref = po.bpla_weights(om[i])
        for a, b in zip(got, ref):
            assert np.array_equal(a, b)


def test_bpla_default_params_are_cli_floats():
    p = ska.BPLAKernel().params
    assert p.kind == 9
    assert p.beta == float(np.float32(0.11)) and p.gap == -8.0 and p.ext == -0.75
    assert p.alpha == 4.5
    assert abs(p.score_table[0] - 5.846613) < 1e-6 and p.score_table[1] == float(np.float32(-1.86))


def _oracle(om, kern, rows, cols):
    return np.array([[po.kernel_value(kern.params.kind, om[i], om[j], kern.params) for j in cols]
                     for i in rows])


@pytest.mark.gpu
@pytest.mark.parametrize("noBP,SW", MODES)
def test_bpla_gram_matches_oracle(gpu_ctx, bpla_set, noBP, SW):
    ds, om = bpla_set
    kern = ska.BPLAKernel(noBP=noBP, SW=SW)
    got = gpu_ctx.gram(ds, kern)
    n = len(om)
    ref = _oracle(om, kern, range(n), range(n))
    up = np.triu_indices(n)
    assert rel_err(got[up], ref[up]) < TOL


@pytest.mark.gpu
def test_bpla_custom_table_and_params(gpu_ctx, bpla_set):
    ds, om = bpla_set
    tb = np.arange(16, dtype=np.float64).reshape(4, 4) / 8.0 - 1.0
    kern = ska.BPLAKernel(gap=-5.0, ext=-1.0, alpha=2.0, beta=0.2, score_table=tb)
    x = np.array([0, 1, 7, 10, 12], np.int32)
    y = np.array([1, 0, 2, 11, 3], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    ref = np.array([po.kernel_value(kern.params.kind, om[a], om[b], kern.params)
                    for a, b in zip(x, y)])
    assert rel_err(got, ref) < TOL


@pytest.mark.gpu
def test_bpla_long_rows_cross_strips(gpu_ctx):
    """L > 128: three 64-row strips and the LDS boundary row twice."""
    seqs = ska.random_sequences(3, 150, 0x5EED0023) + ska.random_sequences(1, 129, 5)
    ds, om = make_examples(seqs)
    for noBP, SW in MODES:
        kern = ska.BPLAKernel(noBP=noBP, SW=SW)
        got = gpu_ctx.gram(ds, kern)
        ref = _oracle(om, kern, range(4), range(4))
        up = np.triu_indices(4)
        assert rel_err(got[up], ref[up]) < TOL


@pytest.mark.gpu
def test_bpla_needs_base_pairs(gpu_ctx):
    """BPLAScore reads p_left/right/unpair; MData(ma) has none (noBP is fine)."""
    ds, om = make_examples(ska.random_sequences(2, 30, 3), use_bp=False)
    with pytest.raises(ska.StemKernelError):
        gpu_ctx.gram(ds, ska.BPLAKernel())
    got = gpu_ctx.gram(ds, ska.BPLAKernel(noBP=True))
    kern = ska.BPLAKernel(noBP=True)
    ref = _oracle(om, kern, range(2), range(2))
    assert rel_err(got, ref) < TOL


@pytest.mark.gpu
def test_bpla_normalized_and_predict(gpu_ctx, bpla_set):
    ds, om = bpla_set
    kern = ska.BPLAKernel()
    g = gpu_ctx.gram(ds, kern, normalize=True)
    assert np.allclose(np.diag(g), 1.0)
    row = gpu_ctx.test_row(ds, 2, ds, kern)
    ref = np.array([po.kernel_value(9, om[i], om[2], kern.params) for i in range(len(om))])
    assert rel_err(row, ref) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("noBP,SW", MODES)
def test_bpla_y_grouped_items(gpu_ctx, bpla_set, noBP, SW, monkeypatch):
    """Many pairs per y: the fast pairs go to the y-grouped kernel (a
    workgroup stages one y for its waves, each wave streams a chunk of
    pairs back to back); the non-dyadic ones (the 3-row alignment) stay on
    the general kernel.  The oracle's values (the chunk sizes and one pair
    per wave: test_bpla_chunk_sizes_agree, experiments build; bit for bit for
    the max-plus SW modes, the exp sums only change order)."""
    ds, om = bpla_set
    n = len(om)
    kern = ska.BPLAKernel(noBP=noBP, SW=SW)
    x = np.tile(np.arange(n, dtype=np.int32), 24)
    y = np.repeat(np.array([0, 11, 12], np.int32), x.size // 3 + 1)[: x.size]
    got = gpu_ctx.pairs(ds, kern, x, y)
    uniq = sorted(set(zip(x.tolist(), y.tolist())))
    ref = {p: po.kernel_value(kern.params.kind, om[p[0]], om[p[1]], kern.params) for p in uniq}
    want = [ref[p] for p in zip(x.tolist(), y.tolist())]
    assert rel_err(got, want) < TOL


@pytest.mark.gpu
@pytest.mark.explib
@pytest.mark.parametrize("noBP,SW", MODES)
def test_bpla_chunk_sizes_agree(gpu_ctx, bpla_set, monkeypatch, noBP, SW):
    """Chunks of 1, 3 and 8 pairs and single-pair launches (experiments
    build: SK_BPLA_CHUNK, SK_BPLA_NO_ITEMS) against the oracle and the
    default chunking."""
    ds, om = bpla_set
    n = len(om)
    kern = ska.BPLAKernel(noBP=noBP, SW=SW)
    x = np.tile(np.arange(n, dtype=np.int32), 24)
    y = np.repeat(np.array([0, 11, 12], np.int32), x.size // 3 + 1)[: x.size]
    got = gpu_ctx.pairs(ds, kern, x, y)
    uniq = sorted(set(zip(x.tolist(), y.tolist())))
    ref = {p: po.kernel_value(kern.params.kind, om[p[0]], om[p[1]], kern.params) for p in uniq}
    want = [ref[p] for p in zip(x.tolist(), y.tolist())]
    for chunk in ("1", "3", "8"):
        monkeypatch.setenv("SK_BPLA_CHUNK", chunk)
        assert rel_err(gpu_ctx.pairs(ds, kern, x, y), want) < TOL
    monkeypatch.delenv("SK_BPLA_CHUNK")
    monkeypatch.setenv("SK_BPLA_NO_ITEMS", "1")
    single = gpu_ctx.pairs(ds, kern, x, y)
    if SW:
        assert np.array_equal(single, got)
    else:
        assert rel_err(single, got) < 1e-13


@pytest.mark.gpu
def test_bpla_chunks_of_long_rows(gpu_ctx):
    """Chunks whose pairs end and start inside a strip, rows of 1 to 3
    strips, a pair of one row after a long one."""
    seqs = ska.random_sequences(2, 150, 0x5EED0033) + ska.random_sequences(2, 64, 9) + \
        ska.random_sequences(2, 100, 11) + ["G", "ACGUACGUAC"]
    ds, om = make_examples(seqs)
    n = len(seqs)
    kern = ska.BPLAKernel()
    x = np.tile(np.array([0, 7, 2, 1, 6, 3, 4, 5], np.int32), 40)
    y = np.repeat(np.array([0, 4], np.int32), x.size // 2)
    got = gpu_ctx.pairs(ds, kern, x, y)
    ref = {(a, b): po.kernel_value(kern.params.kind, om[a], om[b], kern.params)
           for a in range(n) for b in (0, 4)}
    assert rel_err(got, [ref[p] for p in zip(x.tolist(), y.tolist())]) < TOL


@pytest.mark.gpu
def test_bpla_items_workgroup_halved_for_long_rows(gpu_ctx):
    """y-grouped items of long rows: a 16-wave workgroup's LDS (y columns +
    a boundary row per wave) no longer fits a CU, so the engine halves it
    (L = 420: 8 waves; L = 700: 4 waves).  SW modes against the oracle at
    both lengths; the exp sums overflow to inf past a few hundred columns
    as in the reference, so exp mode is compared where it is finite (the
    L = 420 pairs, beta = 0.005) and must be inf where the oracle is."""
    seqs = ska.random_sequences(2, 700, 0x5EED0043) + ska.random_sequences(2, 420, 0x5EED0053)
    ds, om = make_examples(seqs)
    n = len(seqs)
    x = np.tile(np.arange(n, dtype=np.int32), 40)
    for ycols, kern in (((0, 2), ska.BPLAKernel(SW=True)),
                        ((0, 3), ska.BPLAKernel(SW=True, noBP=True)),
                        ((2, 3), ska.BPLAKernel(beta=0.005))):
        y = np.repeat(np.array(ycols, np.int32), x.size // 2)
        got = gpu_ctx.pairs(ds, kern, x, y)
        ref = {(a, b): po.kernel_value(kern.params.kind, om[a], om[b], kern.params)
               for a in range(n) for b in ycols}
        want = np.array([ref[p] for p in zip(x.tolist(), y.tolist())])
        fin = np.isfinite(want)
        assert fin.sum() >= x.size // 4
        assert np.array_equal(np.isinf(got), np.isinf(want))
        assert rel_err(got[fin], want[fin]) < TOL
