"""McCaskill base-pairing probabilities: the engine's GPU
fold (sk_fold_mccaskill, csrc/kernels/fold.hip) in place of the reference's
ViennaRNA pf_fold (common/bpmatrix.cpp:151-177, common/pf_wrapper.cpp:15-36).

Parity against ViennaRNA is unpinned (its parameter files are absent; the
model is the Turner-1999 core).  Pinned here instead:
* the oracle's DP (oracle/fold_oracle.c) equals the Boltzmann sum over every
  secondary structure (exhaustive enumeration) -- Z and every p(i,j) -- for
  random short sequences, with and without --noGU / --noClosingGU /
  --noLonelyPairs (the legacy ViennaRNA pair-type filter, restated);
* the GPU fold equals the oracle's DP (1e-9 absolute on probabilities, 1e-12
  relative on ln Z) up to L = 400, single sequences and batches;
* probabilities are a distribution per base (sum_j p(i,j) <= 1), and the
  threaded dataset builders give the same DAG as the one-at-a-time path.
"""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po


def _rand_seq(rng, L, alphabet="ACGU"):
    return "".join(rng.choice(list(alphabet), L))


@pytest.mark.parametrize("flags", [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 1)])
def test_oracle_dp_equals_enumeration(flags):
    """(no_gu, no_closing_gu, no_lonely_pairs); --noLonelyPairs is ViennaRNA
    1.8's pair-type filter (oracle/fold_oracle.c lonely_filter), under which
    the enumeration sums the structures of the filtered pairs."""
    rng = np.random.default_rng(11 + flags[0] + 2 * flags[1] + 4 * flags[2])
    for _ in range(25):
        s = _rand_seq(rng, int(rng.integers(6, 17)))
        a, pa = po.fold_mccaskill(s, flags[0], flags[1], no_lp=bool(flags[2]))
        b, pb, cnt = po.fold_enum(s, flags[0], flags[1], no_lp=bool(flags[2]))
        assert abs(a - b) < 1e-12 * max(1.0, abs(b)), s
        assert np.max(np.abs(pa - pb), initial=0.0) < 1e-12, s


def test_oracle_enumeration_with_unpairable_characters():
    s = "GGGANNACCCUAGGGNUCCC"
    a, pa = po.fold_mccaskill(s)
    b, pb, cnt = po.fold_enum(s)
    assert cnt > 1 and abs(a - b) < 1e-12 and np.max(np.abs(pa - pb)) < 1e-12


def test_structure_energies():
    # GGGG AAA CCCC: three GC/GC stacks (-330 each) + triloop 570 (dcal/mol)
    assert po.fold_structure_energy("GGGGAAACCCC", "((((...))))") == pytest.approx(-420.0)
    # a hairpin with GU closing is not formed with --noClosingGU
    assert po.fold_structure_energy("GAAAAU", "(....)", no_closing_gu=True) > 1e299


def test_oracle_probabilities_are_per_base_distributions():
    rng = np.random.default_rng(5)
    s = _rand_seq(rng, 120)
    _, p = po.fold_mccaskill(s)
    L = len(s)
    P = np.zeros((L, L))
    P[np.triu_indices(L, 1)] = p
    P = P + P.T
    assert np.all(p >= 0) and np.all(P.sum(1) <= 1 + 1e-12)


def test_threaded_batch_builder_matches_single_adds():
    rng = np.random.default_rng(3)
    seqs = [_rand_seq(rng, 90) for _ in range(5)]
    bpp = [ska.fold(s.lower()) for s in seqs]
    a = ska.Dataset.from_sequences(seqs, bpp=bpp)
    b = ska.Dataset()
    b.add_batch([[s] for s in seqs], [[x] for x in bpp], threads=3)
    for i in range(len(seqs)):
        da, db = a.dag(i), b.dag(i)
        for k in da:
            assert np.array_equal(da[k], db[k]), k


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("flags", [(0, 0), (1, 0), (0, 1)])
def test_gpu_fold_matches_oracle(gpu_ctx, flags):
    rng = np.random.default_rng(100 + flags[0] + 2 * flags[1])
    seqs = [_rand_seq(rng, L) for L in (1, 4, 5, 9, 17, 40, 75, 128, 200, 257, 400)]
    seqs.append("ACGUNNacgut-ggccAAAUUUggcc")
    got, lz = gpu_ctx.fold(seqs, no_gu=bool(flags[0]), no_closing_gu=bool(flags[1]), log_z=True)
    for s, p, z in zip(seqs, got, lz):
        ref_z, ref_p = po.fold_mccaskill(s, *flags)
        assert abs(z - ref_z) <= 1e-12 * max(1.0, abs(ref_z)), (len(s), z, ref_z)
        assert p.shape == ref_p.shape
        assert np.max(np.abs(p - ref_p), initial=0.0) < 1e-9, len(s)


@pytest.mark.gpu
def test_gpu_fold_small_enumeration(gpu_ctx):
    rng = np.random.default_rng(9)
    seqs = [_rand_seq(rng, int(rng.integers(6, 17))) for _ in range(40)]
    got, lz = gpu_ctx.fold(seqs, log_z=True)
    for s, p, z in zip(seqs, got, lz):
        b, pb, _ = po.fold_enum(s)
        assert abs(z - b) < 1e-12 * max(1.0, abs(b)) and np.max(np.abs(p - pb), initial=0.0) < 1e-12


@pytest.mark.gpu
def test_folded_dataset_gram(gpu_ctx):
    """sk_dataset_add_folded (GPU fold + threaded DAG build) gives the same
    Gram as examples built from the oracle-folded bpp, against the kernel
    oracle."""
    rng = np.random.default_rng(21)
    seqs = [_rand_seq(rng, 70) for _ in range(4)]
    ds = ska.Dataset.folded(gpu_ctx, seqs)
    bpp = [po.fold_mccaskill(s.lower())[1] for s in seqs]
    om = [po.OMData([s], [b], 0.01) for s, b in zip(seqs, bpp)]
    p = ska.SuStemStrKernel().params
    ref = np.array([[po.kernel_value(4, om[i], om[j], p) for j in range(4)] for i in range(4)])
    x, y = (a.ravel() for a in np.meshgrid(np.arange(4), np.arange(4), indexing="ij"))
    got = gpu_ctx.pairs(ds, ska.SuStemStrKernel(), x, y).reshape(4, 4)
    assert np.max(np.abs(got - ref) / np.abs(ref)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("no_gu", [False, True])
def test_gpu_fold_no_lonely_pairs(gpu_ctx, no_gu):
    """--noLonelyPairs: the GPU fold equals the restatement with the same
    pair-type filter (which equals enumeration, test above); short ones
    against the enumeration directly, and the filter changes the result."""
    rng = np.random.default_rng(404 + no_gu)
    seqs = [_rand_seq(rng, L) for L in (5, 9, 14, 17, 40, 75, 128, 200, 301)]
    got, lz = gpu_ctx.fold(seqs, no_gu=no_gu, log_z=True, no_lonely_pairs=True)
    plain = gpu_ctx.fold(seqs, no_gu=no_gu)
    for s, p, z, q in zip(seqs, got, lz, plain):
        ref_z, ref_p = po.fold_mccaskill(s, no_gu, False, no_lp=True)
        assert abs(z - ref_z) <= 1e-12 * max(1.0, abs(ref_z)), (len(s), z, ref_z)
        assert np.max(np.abs(p - ref_p), initial=0.0) < 1e-9, len(s)
        if len(s) <= 17:
            b, pb, _ = po.fold_enum(s, no_gu, False, no_lp=True)
            assert abs(z - b) < 1e-12 * max(1.0, abs(b)) and np.max(np.abs(p - pb), initial=0.0) < 1e-12
    assert any(np.max(np.abs(p - q)) > 1e-6 for p, q in zip(got[4:], plain[4:]))


@pytest.mark.gpu
def test_gpu_fold_tables_sized_per_batch(gpu_ctx):
    """the Boltzmann tables are sized by each launch's longest
    sequence (sk_fold_mccaskill builds them per batch), so short sequences
    fold the same -- on the LDS-ring path -- alone and in a call with a
    1,200-nt sequence (no ring; its hairpin / scale tables 19 KB longer); the
    long one against the oracle's ln Z."""
    rng = np.random.default_rng(77)
    short = [_rand_seq(rng, L) for L in (12, 60, 150)]
    long_ = _rand_seq(rng, 1200)
    a, za = gpu_ctx.fold(short, log_z=True)
    b, zb = gpu_ctx.fold(short + [long_], log_z=True)
    for k in range(len(short)):
        assert np.max(np.abs(a[k] - b[k]), initial=0.0) < 1e-13 and abs(za[k] - zb[k]) <= 1e-13 * abs(za[k])
    ref_z, _ = po.fold_mccaskill(long_, 0, 0)
    assert abs(zb[-1] - ref_z) <= 1e-12 * abs(ref_z)
