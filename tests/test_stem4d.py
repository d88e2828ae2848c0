"""4-D stem kernel (stem_kernel/): oracle anchors on CPU,
HIP parity (1e-6 relative, double) on the GPU.

Parity anchors: the reference's CLI default without Vienna runs
NormalBasePair with bp_bound 1.0, which makes every kernel value 1
(SURVEY.md §8c probe anchor); the -p path (bp_model 0) uses the dataset's
base-pairing probabilities.  Sequences are lowercased as the reference loader
does (common/example.cpp:26-34)."""
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
                             p.subst, p.bp_bound, p.bp_model, p.loop, p.len_band, p.ali_bound,
                             p.ali_zerop_fixed))
    return np.array(out)


def test_oracle_normal_basepair_is_one():
    s = [q.lower() for q in ska.random_sequences(3, 25, 11)]
    for a in s:
        for b in s:
            assert po.stem4d(a, None, b, None, bp_bound=1.0, model=1) == 1.0
            assert po.stem4d(a, None, b, None, bp_bound=1.0, model=2) == 1.0


@pytest.mark.parametrize("model,bound", [(0, 0.0), (0, 0.2), (1, 0.5), (2, 0.5), (1, 1.0)])
def test_oracle_ksum_equals_chain(model, bound):
    """The K-sum identity behind the engine's full_dp kernel:
    K0(0,n,0,m) of the reference's K0..K3 chain (stem_kernel.cpp:282-351,
    restated in the oracle) equals 1 + the sum of the stacking sources, up to
    the association of non-negative terms -- lengths 0, 1, short and ragged."""
    s = ska.random_sequences(3, 23, 71) + ska.random_sequences(2, 9, 72) + ["", "c", "GGGAAACCC"]
    for a in s:
        for b in s:
            xa, xb = a.lower(), b.lower()
            bx = ska.fold(a) if a else np.zeros(0)
            by = ska.fold(b) if b else np.zeros(0)
            args = (xa, bx if model == 0 else None, xb, by if model == 0 else None, 0.7, 1.3, 0.4,
                    bound, model, 3)
            chain, ksum = po.stem4d(*args), po.stem4d_ksum(*args)
            assert abs(chain - ksum) <= 1e-13 * abs(chain), (a, b, chain, ksum)


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
def test_stem4d_col_default_oracle(gpu_ctx):
    """The default full_dp kernel (the column-group kernel for |y| < 512)
    against the oracle on short sequences, CPL 1-4, empty and one-residue
    sequences included (the variant comparisons: the explib test below)."""
    seqs = _seqs() + ["", "G"] + ska.random_sequences(2, 130, 0x5EED0043)
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D()
    a = gpu_ctx.gram(ds, kern)
    assert gpu_ctx.last_classes()["stem4d_col"]
    n = len(seqs)
    iu = list(zip(*np.triu_indices(n)))
    ref = _oracle(seqs, kern, iu)
    assert rel_err(a[tuple(np.array(iu).T)], ref) < TOL
    assert a[n - 4, n - 4] == 1.0 and np.all(a[n - 4, :] == 1.0)  # the empty sequence: K = 1


@pytest.mark.gpu
@pytest.mark.explib
@pytest.mark.parametrize("mode", ["pre", "col", "ksum"])
def test_stem4d_ksum_equals_four_state(gpu_ctx, monkeypatch, mode):
    """full_dp with the K chain summed (K0(0,n,0,m) = 1 + the sum of every
    stacking source) against the four-state planes
    (SK4_NO_GSUM=1): equal up to the association of non-negative sums, CPL
    1-4, empty and one-residue sequences included, both against the oracle.
    "col" runs the column-group kernel (sk_stem4d_col_kernel, the default for
    |y| < 512), "pre" the pre-combined span kernel (sk_stem4d_pre_kernel,
    SK4_SPAN=1), "ksum" the K-sum span kernel (sk_stem4d_gsum_kernel) on the
    same short sequences (SK4_NO_PRE=1)."""
    seqs = _seqs() + ["", "G"] + ska.random_sequences(2, 130, 0x5EED0043)
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D()
    if mode == "ksum":
        monkeypatch.setenv("SK4_NO_PRE", "1")
    if mode == "pre":
        monkeypatch.setenv("SK4_SPAN", "1")
    a = gpu_ctx.gram(ds, kern)
    assert bool(gpu_ctx.last_classes()["stem4d_col"]) == (mode == "col")
    monkeypatch.setenv("SK4_NO_GSUM", "1")
    b = gpu_ctx.gram(ds, kern)
    assert rel_err(a, b) < 1e-12
    n = len(seqs)
    iu = list(zip(*np.triu_indices(n)))
    ref = _oracle(seqs, kern, iu)
    assert rel_err(a[tuple(np.array(iu).T)], ref) < TOL
    assert a[n - 4, n - 4] == 1.0 and np.all(a[n - 4, :] == 1.0)  # the empty sequence: K = 1


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


@pytest.mark.gpu
def test_stem4d_resident_tables_two_datasets(gpu_ctx):
    """The per-example tables stay resident per dataset (sk_api.cpp
    stem4d_dataset_tables): test x train across two datasets reads each side
    from its own dataset's tables, and a new bp model or loop rebuilds them
    (the same datasets first under NormalBasePair loop 3, then -p, then
    WobbleBasePair loop 5)."""
    tr = ska.random_sequences(4, 45, 0x5EED0051) + ["GGGGAAAACCCC"]
    te = ska.random_sequences(3, 70, 0x5EED0052)
    dtr, _ = make_examples(tr)
    dte, _ = make_examples(te)
    for kern in [ska.StemKernel4D(bp_model=1, bp_bound=0.5), ska.StemKernel4D(),
                 ska.StemKernel4D(bp_model=2, bp_bound=0.5, loop=5)]:
        got, _ = gpu_ctx.test_matrix(dte, dtr, kern)
        p = kern.params
        ref = np.array([[po.stem4d(a.lower(), ska.fold(a), b.lower(), ska.fold(b), p.gap, p.stack,
                                   p.subst, p.bp_bound, p.bp_model, p.loop, p.len_band,
                                   p.ali_bound, p.ali_zerop_fixed) for b in tr] for a in te])
        assert rel_err(got, ref) < TOL


@pytest.mark.gpu
def test_stem4d_col_cpl8_matches_oracle(gpu_ctx):
    """The column kernel's widest class (CPL 8: 256 <= |y| < 512, one k
    tile, NB 1) against the oracle: short x, long y (the oracle's cost is
    |x|^2 |y|^2 / 4 cells), y's of different lengths in one batch (W from the
    shortest)."""
    xs = ska.random_sequences(2, 24, 0x5EED0061) + ["GGGCGCAAGCCU"]
    ys = ska.random_sequences(1, 300, 0x5EED0062) + ska.random_sequences(1, 457, 0x5EED0063)
    seqs = xs + ys
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(bp_model=2, bp_bound=0.3)
    x = np.array([0, 1, 2, 0, 2], np.int32)
    y = np.array([3, 3, 4, 4, 3], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    assert gpu_ctx.last_classes()["stem4d_col"] == [8]
    ref = _oracle(seqs, kern, list(zip(x, y)))
    assert rel_err(got, ref) < TOL


@pytest.mark.gpu
def test_stem4d_short_y_limits(gpu_ctx):
    """y lengths 2 .. 8 around the column kernel's limit W <= m - PF - 2: the
    shortest go to the span kernel in batches of their own (run_stem4d), the
    next run one to a few waves; every pair against the oracle."""
    ys = ["GC", "GCU", "GGCC", "GAUCA", "GGAUCC", "GGGAUCC", "GCGAAAGC"]
    xs = ska.random_sequences(3, 16, 0x5EED0071) + ["GGGGAAACCCC"]
    seqs = xs + ys
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(bp_model=2, bp_bound=0.3)
    pairs = [(a, len(xs) + b) for a in range(len(xs)) for b in range(len(ys))]
    x = np.array([p[0] for p in pairs], np.int32)
    y = np.array([p[1] for p in pairs], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    ref = _oracle(seqs, kern, pairs)
    assert rel_err(got, ref) < TOL


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


# ---------------------------------------------------------------- -a option
def _indel_variants(seed, n, L):
    """Related sequences (substitutions, insertions, deletions) so that the
    PairHMM MAP path leaves the diagonal and anchors are sparse."""
    rng = np.random.default_rng(seed)
    base = ska.random_sequences(1, L, seed)[0]
    out = [base]
    for _ in range(n - 1):
        r = []
        for c in base:
            u = rng.random()
            if u < 0.06:
                continue
            r.append("ACGU"[rng.integers(4)] if u < 0.2 else c)
            if rng.random() < 0.06:
                r.append("ACGU"[rng.integers(4)])
        out.append("".join(r))
    return out


def test_isinf_bool_makes_zerop_false(tmp_path):
    """LogValue's zerop is `std::isinf(x.log())<0` (stem_kernel/log_value.h:374-378).
    Built with a C++11 <cmath> (as g++ builds the reference today) std::isinf
    returns bool, so the test is false even for log(0): the basis of
    ali_zerop_fixed = 0.  Compiles the expression itself (not reference code)."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ absent")
    src = tmp_path / "z.cpp"
    src.write_text("#include <cmath>\n#include <cstdio>\n#include <limits>\n"
                   "int main(){double v=-std::numeric_limits<double>::infinity();"
                   "std::printf(\"%d\", (int)(std::isinf(v)<0));}\n")
    exe = tmp_path / "z"
    subprocess.run([gxx, "-std=gnu++17", "-w", str(src), "-o", str(exe)], check=True)
    assert subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout == "0"


def test_oracle_phmm_posteriors():
    """zerop_fixed: posteriors are a distribution over each residue's state
    (every x residue is emitted once, in M or IX; every y residue in M or IY),
    up to the probcons log1exp0 approximation.  As built today (0): NaN."""
    x, y = [s.lower() for s in _indel_variants(5, 2, 45)]
    fb = po.phmm_posterior(x, y, 1)
    assert np.all(np.isfinite(fb)) and fb.min() >= 0.0
    mx = fb[0, 1:, :].sum(1) + fb[1, 1:, :].sum(1)
    my = fb[0, :, 1:].sum(0) + fb[2, :, 1:].sum(0)
    assert np.abs(mx - 1).max() < 1e-3 and np.abs(my - 1).max() < 1e-3
    assert np.all(np.isnan(po.phmm_posterior(x, y, 0)))
    with pytest.raises(ValueError):
        po.phmm_posterior("acgt", "acgu", 1)


@pytest.mark.parametrize("band", [0, 2, 5])
def test_oracle_alignment_constraints_shape(band):
    """Constraints are monotone (the 4-D kernel's boundary reads rely on it),
    inside [0, |y|], anchor rows are single points when band == 0, and the
    NaN posteriors of zerop_fixed = 0 leave the whole range."""
    seqs = [s.lower() for s in _indel_variants(7, 4, 50)] + ["acgu", "a"]
    for x in seqs:
        for y in seqs:
            for ab in (0.2, 0.5, 0.9):
                lo, hi = po.alignment_constraints(x, y, ab, band, 1)
                assert np.all(lo <= hi) and hi.max() <= len(y)
                assert np.all(np.diff(lo.astype(int)) >= 0) and np.all(np.diff(hi.astype(int)) >= 0)
                if band == 0 and len(x) > 10 and x[:10] == y[:10]:
                    assert (lo == hi).sum() > len(x) // 2
                lo0, hi0 = po.alignment_constraints(x, y, ab, band, 0)
                assert np.all(lo0 == 0) and np.all(hi0 == len(y))
    # band alone (ali_bound 0) is the -b diagonal band
    lo, hi = po.alignment_constraints(seqs[0], seqs[1], 0.0, 3, 1)
    lo2, hi2 = np.zeros_like(lo), np.zeros_like(hi)
    po.oracle().orc_stem4d_band(len(seqs[0]), len(seqs[1]), 3,
                                lo2.ctypes.data_as(po._U), hi2.ctypes.data_as(po._U))
    assert np.array_equal(lo, lo2) and np.array_equal(hi, hi2)


def test_oracle_ali_as_built_equals_full_dp():
    """zerop_fixed = 0: the NaN posteriors anchor nothing, the constraints are
    the full range whatever the band, and partial_dp over the full range is
    full_dp bit for bit -- what the engine runs for this mode."""
    seqs = _indel_variants(3, 3, 22) + ["acgu", "a"]
    for a in seqs:
        for b in seqs:
            full = po.stem4d(a.lower(), ska.fold(a), b.lower(), ska.fold(b))
            for band in (0, 2, 5):
                k0 = po.stem4d(a.lower(), ska.fold(a), b.lower(), ska.fold(b), ali_bound=0.5,
                               band=band)
                assert k0 == full


@pytest.mark.gpu
@pytest.mark.parametrize("fixed,ab,band", [(1, 0.5, 0), (1, 0.8, 0), (1, 0.3, 4), (0, 0.5, 0),
                                           (0, 0.5, 3)])
def test_stem4d_alignment_constraints_match_oracle(gpu_ctx, fixed, ab, band):
    """-a: PairHMM posteriors, MAP path and anchors on the GPU, then
    partial_dp over them, against the oracle (1e-6 relative)."""
    seqs = _indel_variants(11, 5, 48) + _indel_variants(12, 2, 30) + ["GGGAAACCC", "A"]
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(ali_bound=ab, ali_zerop_fixed=fixed, band=band)
    n = len(seqs)
    iu = list(zip(*np.triu_indices(n)))
    got = gpu_ctx.gram(ds, kern)
    ref = _oracle(seqs, kern, iu)
    assert rel_err(got[tuple(np.array(iu).T)], ref) < TOL
    x = np.array([5, 0, 7, 8, 2], np.int32)
    y = np.array([0, 5, 1, 3, 8], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    assert rel_err(got, _oracle(seqs, kern, list(zip(x, y)))) < TOL


@pytest.mark.gpu
def test_stem4d_alignment_constraints_reject_non_acgu(gpu_ctx):
    ds, _ = make_examples(["ACGUNACGU", "ACGUACGU"])
    with pytest.raises(ska.StemKernelError):
        gpu_ctx.gram(ds, ska.StemKernel4D(ali_bound=0.5))
    gpu_ctx.gram(ds, ska.StemKernel4D())  # without -a the residues are free


@pytest.mark.gpu
@pytest.mark.parametrize("band", [0, 4])
def test_stem4d_alignment_constraints_long(gpu_ctx, band):
    """Sequences past 64 and 128 nt: several 64-row strips of the PairHMM
    sweep and the 4-slot register class of the 4-D kernel, with anchored
    constraints (oracle fast: partial_dp only visits constrained cells)."""
    seqs = _indel_variants(21, 3, 150) + _indel_variants(22, 2, 75)
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(ali_bound=0.5, ali_zerop_fixed=True, band=band)
    x = np.array([0, 1, 2, 0, 3, 4, 1], np.int32)
    y = np.array([1, 0, 2, 2, 4, 3, 3], np.int32)
    got = gpu_ctx.pairs(ds, kern, x, y)
    assert rel_err(got, _oracle(seqs, kern, list(zip(x, y)))) < TOL


@pytest.mark.gpu
@pytest.mark.explib
@pytest.mark.parametrize("band", [0, 5])
def test_stem4d_stream_parts_identical(gpu_ctx, band, monkeypatch):
    """A batch's pairs dealt to 1-4 parts whose span launches run on their own
    streams (SK4_STREAMS): every value bit-identical (each pair's planes are
    computed by the same waves in the same order whatever the part), and each
    span launch timed by its own events (sk_last_launch_ms)."""
    seqs = _seqs()
    ds, _ = make_examples(seqs)
    kern = ska.StemKernel4D(band=band)
    base = None
    for parts in (1, 2, 3, 4):
        monkeypatch.setenv("SK4_STREAMS", str(parts))
        got = gpu_ctx.gram(ds, kern)
        lm = gpu_ctx.last_launch_ms()
        assert lm["launches"] >= 1 and lm["ms_sum"] > 0.0
        if base is None:
            base = got
        else:
            assert np.array_equal(got, base)
