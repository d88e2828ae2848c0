"""Randomized parity sweep: seeded random sequence sets (lengths 12-260, so
the DAG stem register classes MAXK 4-24 and the profile string kernel's 1-5
strips), random thresholds and random kernel parameters (beta, loop_gap,
gap, alpha, the length band including 0 = off), every kind 0-7, every
ordered pair (the stem kernels are asymmetric), the HIP engine through the C
ABI against the oracle (oracle/pyoracle.py kernel_value, def_kernel.h:113-190
composition).  Tolerance: 1e-6 relative (BASELINE.json north_star, double).
"""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, rel_err

TOL = 1e-6
SEEDS = [11, 23, 37, 58, 71, 86, 94, 105]


def _case(seed):
    rng = np.random.default_rng(seed)
    lens = [int(v) for v in rng.integers(12, 261, 6)]
    seqs = [ska.random_sequences(1, n, seed * 100 + i)[0] for i, n in enumerate(lens)]
    th = float(rng.choice([0.01, 0.02, 0.05]))
    p = dict(alpha=float(rng.uniform(0.05, 0.5)), beta=float(rng.uniform(0.1, 0.8)),
             loop_gap=float(rng.uniform(0.05, 0.6)), gap=float(rng.uniform(0.3, 0.95)),
             len_band=int(rng.choice([0, 1, 4, 10, 30])))
    stem = dict(beta=p["beta"], loop_gap=p["loop_gap"], len_band=p["len_band"])
    # the simple score's stack / covariance weights and string mismatch
    si = dict(loop_gap=p["loop_gap"], stack=float(rng.uniform(0.8, 2.0)), covar=float(rng.uniform(0.3, 1.2)),
              len_band=p["len_band"])
    mm = float(rng.uniform(0.2, 0.9))
    kernels = [ska.SuStemKernel(**stem), ska.SiStemKernel(**si),
               ska.StringKernel(gap=p["gap"], alpha=p["alpha"]),
               ska.StringKernel(gap=p["gap"], match=1.0, mismatch=mm),
               ska.SuStemStrKernel(**p), ska.SiStemStrKernel(**si, gap=p["gap"], match=1.0, mismatch=mm),
               ska.LSuStemKernel(**stem), ska.LSuStemStrKernel(**p)]
    return seqs, th, kernels


def test_sweep_cases_are_distinct():
    """CPU: the seeds give different sizes and parameters (the sweep is not
    one case repeated)."""
    cases = [_case(s) for s in SEEDS]
    assert len({tuple(len(q) for q in c[0]) for c in cases}) == len(SEEDS)
    assert len({c[2][0].params.len_band for c in cases}) > 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_sweep(gpu_ctx, seed):
    seqs, th, kernels = _case(seed)
    ds, om = make_examples(seqs, th=th)
    n = len(seqs)
    x, y = (a.ravel() for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
    for kern in kernels:
        got = gpu_ctx.pairs(ds, kern, x, y).reshape(n, n)
        ref = np.array([[po.kernel_value(kern.params.kind, om[i], om[j], kern.params) for j in range(n)]
                        for i in range(n)])
        assert rel_err(got, ref) < TOL, (seed, kern.params.kind)
