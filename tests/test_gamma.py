"""Gamma and phi rows of the DAG stem kernel (dag_stem.hip):
x loop rows with one bp-frequency entry and no gap column are not swept per
pair, their G0 rows come from the y's Gamma table; stem rows whose children
are all such rows are combinations of the y's Phi and Gamma rows.  The
schedules with both (default), without phi rows (SK_NO_PHI), without
either (SK_NO_GAMMA), with every read row stored (SK_STORE_ALL: by default a
row read only by the next one stays in registers) and in the reference
numbering (SK_REF_ORDER: by default a depth-first order; all four read when a
dataset is packed, in the experiments build only: test_gamma_switches_agree
runs under tests/test_explib.py) agree to rounding,
and the default matches the oracle, on inputs that mix the cases: single sequences,
gapless alignments (several bp-frequency entries per node: the general
seeds), gapped alignments (no Gamma / Phi for that y), length bands and
separate row / column sets."""
import os

import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, mutate_alignment, rel_err

pytestmark = pytest.mark.gpu


def _inputs(seed):
    base = ska.random_sequences(4, 64, seed)
    return [base[0], mutate_alignment(base[1], 3, seed + 1, gap=0.0),
            mutate_alignment(base[2], 2, seed + 2), base[3],
            mutate_alignment(base[0], 2, seed + 3, gap=0.0)]


def _gram(ctx, items, kern, switch=None):
    saved = {k: os.environ.pop(k, None) for k in ("SK_NO_GAMMA", "SK_NO_PHI", "SK_STORE_ALL", "SK_REF_ORDER")}
    try:
        if switch:
            os.environ[switch] = "1"
        ds, om = make_examples(items)
        return ctx.gram(ds, kern), om
    finally:
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


@pytest.mark.parametrize("band", [0, 4])
def test_gamma_oracle(gpu_ctx, band):
    items = _inputs(0x6A44A + band)
    kern = ska.SuStemKernel(loop_gap=0.4, len_band=band)
    on, om = _gram(gpu_ctx, items, kern)
    lm = gpu_ctx.last_launch_ms()
    assert lm["launches"] >= 1 and lm["ms_sum"] > 0.0
    n = len(items)
    ref = np.array([[po.su_stem(om[i], om[j], 0.4, kern.params.beta, band) for j in range(n)]
                    for i in range(n)])
    up = np.triu_indices(n)
    assert rel_err(on[up], ref[up]) < 1e-6


@pytest.mark.explib
@pytest.mark.parametrize("band", [0, 4])
def test_gamma_switches_agree(gpu_ctx, band):
    """The schedules agree to rounding (experiments build: SK_NO_PHI,
    SK_NO_GAMMA, SK_STORE_ALL, SK_REF_ORDER are read when a dataset is
    packed)."""
    items = _inputs(0x6A44A + band)
    kern = ska.SuStemKernel(loop_gap=0.4, len_band=band)
    on, _ = _gram(gpu_ctx, items, kern)
    no_phi, _ = _gram(gpu_ctx, items, kern, "SK_NO_PHI")
    off, _ = _gram(gpu_ctx, items, kern, "SK_NO_GAMMA")
    stored, _ = _gram(gpu_ctx, items, kern, "SK_STORE_ALL")
    ref_order, _ = _gram(gpu_ctx, items, kern, "SK_REF_ORDER")
    assert rel_err(on, off) < 1e-12 and rel_err(no_phi, off) < 1e-12 and rel_err(on, stored) < 1e-14
    assert rel_err(on, ref_order) < 1e-12


def test_gamma_row_and_column_sets(gpu_ctx):
    """Gamma and phi keys belong to the row (x) set; the column set's Gamma
    and Phi tables are built from them."""
    train, om = make_examples(_inputs(0x6A450))
    test, omt = make_examples([ska.random_sequences(1, 70, 0x6A451)[0],
                               mutate_alignment(ska.random_sequences(1, 66, 0x6A452)[0], 2, 3, gap=0.0)])
    kern = ska.SuStemKernel()
    for t in range(2):
        row = gpu_ctx.test_row(test, t, train, kern)
        ref = [po.su_stem(om[x], omt[t]) for x in range(len(om))]
        assert rel_err(row, ref) < 1e-6
