"""Pin the oracle (and the product tables) to the reference itself.

oracle/_ref/libskref.so is the reference's own common/rna.cpp,
common/profile.cpp and stem_kernel_lite/ribosum.cpp, compiled unmodified from
/root/reference by oracle/Makefile (the only hot-path translation units that
build with nothing but the C++ standard library).  The DP kernels themselves
cannot be built here (Boost, ViennaRNA, config.h): see DESIGN.md §Oracle.
"""
import ctypes as C

import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import pyoracle as po

ref = po.reference_partial()
needs_ref = pytest.mark.skipif(ref is None, reason="oracle/_ref not built (reference absent)")


def _tables(fn):
    s = np.zeros(16, np.float32)
    p = np.zeros(256, np.float32)
    fn(s.ctypes.data_as(po._F), p.ctypes.data_as(po._F))
    return s, p


@needs_ref
def test_ribosum_tables_match_reference():
    rs, rp = _tables(ref.skref_ribosum)
    os_, op = _tables(po.oracle().orc_ribosum_tables)
    ls, lp = _tables(ska.lib().sk_ribosum_tables)
    assert np.array_equal(rs, os_) and np.array_equal(rp, op)
    assert np.array_equal(rs, ls) and np.array_equal(rp, lp)


@needs_ref
def test_char2rna_matches_reference():
    for c in range(1, 256):
        r = ref.skref_char2rna(c)
        assert po.oracle().orc_char2rna(c) == r, chr(c)
        assert ska.lib().sk_char2rna(c) == r, chr(c)


@needs_ref
@pytest.mark.parametrize("seed", range(6))
def test_profile_matches_reference(seed):
    rng = np.random.default_rng(seed)
    alphabet = list("ACGUTacgut-RYMKSWBDHVNrymkswbdhvn.X")
    L = int(rng.integers(1, 60))
    rows = ["".join(rng.choice(alphabet, size=L)) for _ in range(int(rng.integers(1, 5)))]
    out = np.zeros((L, 5), np.float32)
    ns = C.c_float()
    arr = (C.c_char_p * len(rows))(*[r.encode() for r in rows])
    assert ref.skref_profile(len(rows), arr, out.ctypes.data_as(po._F), C.byref(ns)) == L
    om = po.OMData(rows, None, use_bp=False)
    o = np.zeros((L, 5), np.float32)
    ons = C.c_float()
    po.oracle().orc_mdata_profile(om.h, o.ctypes.data_as(po._F), C.byref(ons))
    assert np.array_equal(out, o) and ns.value == ons.value
    ds = ska.Dataset()
    ds.add("+1", rows, use_bp=False)
    prof, pns = ds.profile(0)
    assert np.array_equal(out, prof) and ns.value == pns
