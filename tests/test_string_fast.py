"""Profile string kernel fast path (profile_string.hip: dyadic, never-empty
profiles, both examples weighted or neither): the oracle's values, and the
general kernel's (SK_STR_GENERAL=1) to rounding, on inputs that mix the
cases — single sequences and IUPAC codes (fast), 2- and 4-row alignments
(dyadic: fast), a 3-row alignment and an all-gap column (general), lengths
below one strip, at strip boundaries and over three strips, weighted (bpp)
and unweighted (no bp information) examples."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, mutate_alignment, rel_err

pytestmark = pytest.mark.gpu


def _items():
    s = ska.random_sequences(6, 150, 0x5EED0B00)
    return [s[0], s[1][:64], s[2][:65], s[3][:20], "ACGUNRYKMSWACGUACGGGAAACCCRY",
            mutate_alignment(s[4][:90], 2, 5, gap=0.0), mutate_alignment(s[5][:130], 4, 6),
            mutate_alignment(s[4][:70], 3, 7), ["ACG-UAGC", "ACG-UUGC"], s[2][:129]]


@pytest.mark.parametrize("use_bp", [True, False])
def test_string_fast_matches_oracle(gpu_ctx, use_bp):
    items = _items()
    ds, om = make_examples(items, use_bp=use_bp)
    n = len(items)
    for kern in (ska.StringKernel(gap=0.8, alpha=0.2), ska.StringKernel(gap=0.7, match=1.0, mismatch=0.6)):
        got = gpu_ctx.gram(ds, kern)
        ref = np.array([[po.kernel_value(kern.params.kind, om[i], om[j], kern.params) for j in range(n)]
                        for i in range(n)])
        up = np.triu_indices(n)
        assert rel_err(got[up], ref[up]) < 1e-6


@pytest.mark.explib
@pytest.mark.parametrize("use_bp", [True, False])
def test_string_fast_equals_general(gpu_ctx, use_bp, monkeypatch):
    """The fast paths against the general kernel on the same pairs
    (experiments build: SK_STR_GENERAL)."""
    items = _items()
    ds, om = make_examples(items, use_bp=use_bp)
    for kern in (ska.StringKernel(gap=0.8, alpha=0.2), ska.StringKernel(gap=0.7, match=1.0, mismatch=0.6)):
        got = gpu_ctx.gram(ds, kern)
        monkeypatch.setenv("SK_STR_GENERAL", "1")
        gen = gpu_ctx.gram(ds, kern)
        monkeypatch.delenv("SK_STR_GENERAL")
        assert rel_err(got, gen) < 1e-12


def test_string_fast_mixed_weights_and_sets(gpu_ctx):
    """A weighted row set against an unweighted column set (the general
    kernel's no-weights rule for such pairs) and a sum kernel over both."""
    a = ska.random_sequences(3, 80, 0x5EED0B10)
    b = ska.random_sequences(2, 70, 0x5EED0B11)
    dw, omw = make_examples(a)
    du, omu = make_examples(b, use_bp=False)
    kern = ska.StringKernel()
    m, _ = gpu_ctx.test_matrix(du, dw, kern)
    ref = np.array([[po.kernel_value(kern.params.kind, omw[j], omu[i], kern.params) for j in range(3)]
                    for i in range(2)])
    assert rel_err(m, ref) < 1e-6
    ss = ska.SuStemStrKernel()
    got = gpu_ctx.gram(dw, ss)
    ref = np.array([[po.kernel_value(ss.params.kind, omw[i], omw[j], ss.params) for j in range(3)]
                    for i in range(3)])
    assert rel_err(got[np.triu_indices(3)], ref[np.triu_indices(3)]) < 1e-6
