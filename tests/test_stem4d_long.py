"""4-D stem kernel beyond one 512-cell k tile (|y| >= 512: the y spans of a
plane are swept tile by tile, right to left, stem4d.hip) and with a long x.
The reference's full_dp / partial_dp have no length limit
(stem_kernel/stem_kernel.cpp:113-351).  Fixtures: tests/golden/make_golden_4d_long.py
(CPU oracle).  Tolerance 1e-6 relative."""
import hashlib
import os

import numpy as np
import pytest

import stem_kernel_amd as ska
from tests.helpers import rel_err

TOL = 1e-6
LONG = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "long_4d.npz"))


def _cases():
    return [(str(a), str(b), int(c)) for a, b, c in zip(LONG["x"], LONG["y"], LONG["band"])]


def test_fold_bytes_pinned():
    h = hashlib.sha256()
    for a, b, _ in _cases():
        for t in (a, b):
            h.update(np.ascontiguousarray(ska.fold(t.lower()), np.float64).tobytes())
    assert h.hexdigest() == str(LONG["sha"])


def test_cases_cross_tiles():
    assert max(len(b) for _, b, _ in _cases()) + 1 > 2 * 512
    assert any(512 <= len(b) < 1023 for _, b, _ in _cases())


@pytest.fixture(scope="module")
def long_set():
    seqs = sorted({s for a, b, _ in _cases() for s in (a, b)})
    ds = ska.Dataset.from_sequences(seqs, bpp=[ska.fold(s.lower()) for s in seqs])
    return ds, {s: i for i, s in enumerate(seqs)}


@pytest.mark.gpu
def test_stem4d_long_one_call_per_pair(gpu_ctx, long_set):
    ds, idx = long_set
    for k, (a, b, band) in enumerate(_cases()):
        got = gpu_ctx.pairs(ds, ska.StemKernel4D(band=band), [idx[a]], [idx[b]])
        assert rel_err(got, LONG["value"][k:k + 1]) < TOL, (k, got, LONG["value"][k])
        assert gpu_ctx.last_classes()["stem4d"] == [(8 if len(b) >= 256 else 1, band > 0)]


@pytest.mark.gpu
def test_stem4d_long_mixed_call(gpu_ctx, long_set):
    """Full-DP pairs of every length in one call: the call's class follows
    its longest y (CPL 8, 3 tiles), short y's run one tile of it."""
    ds, idx = long_set
    cs = [(k, c) for k, c in enumerate(_cases()) if c[2] == 0]
    got = gpu_ctx.pairs(ds, ska.StemKernel4D(), [idx[a] for _, (a, _, _) in cs],
                        [idx[b] for _, (_, b, _) in cs])
    assert rel_err(got, LONG["value"][[k for k, _ in cs]]) < TOL


LONGX = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "longx_4d.npz"))


def _cases_x():
    return [(str(a), str(b)) for a, b in zip(LONGX["x"], LONGX["y"])]


def test_longx_fold_bytes_pinned():
    h = hashlib.sha256()
    for a, b in _cases_x():
        for t in (a, b):
            h.update(np.ascontiguousarray(ska.fold(t.lower()), np.float64).tobytes())
    assert h.hexdigest() == str(LONGX["sha"])
    assert max(len(a) for a, _ in _cases_x()) > 2048  # one pair past the column kernel's x limit
    assert any(512 < len(a) <= 2048 for a, _ in _cases_x())


@pytest.mark.gpu
def test_stem4d_long_x_short_y(gpu_ctx):
    """Long x against short y: the column kernel's x characters
    sit in LDS sized from the batch's longest x, so |x| 640 / 700 / 1,200
    against |y| 40-100 run on it (before, a fixed 512-byte region dropped the
    tail of x); |x| = 2,100 is past its limit and runs the span kernel.  One
    call per pair and one call for all; every value against the oracle's."""
    seqs = sorted({s for c in _cases_x() for s in c})
    ds = ska.Dataset.from_sequences(seqs, bpp=[ska.fold(s.lower()) for s in seqs])
    idx = {s: i for i, s in enumerate(seqs)}
    for k, (a, b) in enumerate(_cases_x()):
        got = gpu_ctx.pairs(ds, ska.StemKernel4D(), [idx[a]], [idx[b]])
        assert rel_err(got, LONGX["value"][k:k + 1]) < TOL, (k, got, LONGX["value"][k])
        cls = gpu_ctx.last_classes()
        if len(a) <= 2048:  # (stem4d lists the column kernel's classes too)
            assert cls["stem4d_col"] and cls["stem4d"] == [(c, False) for c in cls["stem4d_col"]], (k, cls)
        else:
            assert cls["stem4d"] and not cls["stem4d_col"], (k, cls)
    cs = _cases_x()
    got = gpu_ctx.pairs(ds, ska.StemKernel4D(), [idx[a] for a, _ in cs], [idx[b] for _, b in cs])
    assert rel_err(got, LONGX["value"]) < TOL
