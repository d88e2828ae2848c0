"""ctypes loader for the CPU ORACLE (oracle/liboracle.so) and the partial
reference build (oracle/_ref/libskref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker, never as the product.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libskref.so")

_o = None
_r = None

_D = C.POINTER(C.c_double)
_U = C.POINTER(C.c_uint32)
_F = C.POINTER(C.c_float)


def oracle():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"{ORACLE_SO} not built (make -C oracle)")
        L = C.CDLL(ORACLE_SO)
        L.orc_mdata_new.restype = C.c_void_p
        L.orc_mdata_new.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(_D), C.c_float, C.c_int]
        L.orc_mdata_free.argtypes = [C.c_void_p]
        for n in ("orc_mdata_n_nodes", "orc_mdata_n_edges", "orc_mdata_n_bpfreq",
                  "orc_mdata_seq_len", "orc_mdata_n_roots"):
            getattr(L, n).argtypes = [C.c_void_p]
            getattr(L, n).restype = C.c_int
        L.orc_mdata_nodes.argtypes = [C.c_void_p, _U, _U, _U, _U, _F, _U]
        L.orc_mdata_edges.argtypes = [C.c_void_p, _U, _U]
        L.orc_mdata_bpfreq.argtypes = [C.c_void_p, _U, _F]
        L.orc_mdata_roots.argtypes = [C.c_void_p, _U]
        L.orc_mdata_weight.argtypes = [C.c_void_p, _F]
        L.orc_mdata_profile.argtypes = [C.c_void_p, _F, _F]
        L.orc_mdata_bpp.argtypes = [C.c_void_p, _D]
        for n in ("orc_su_stem",):
            getattr(L, n).restype = C.c_double
            getattr(L, n).argtypes = [C.c_void_p, C.c_void_p, C.c_double, C.c_double, C.c_uint]
        L.orc_si_stem.restype = C.c_double
        L.orc_si_stem.argtypes = [C.c_void_p, C.c_void_p, C.c_double, C.c_double, C.c_double, C.c_uint]
        L.orc_profile_string.restype = C.c_double
        L.orc_profile_string.argtypes = [C.c_void_p, C.c_void_p, C.c_double, C.c_int, C.c_double,
                                         C.c_double, C.c_double]
        L.orc_ribosum_tables.argtypes = [_F, _F]
        L.orc_char2rna.argtypes = [C.c_int]
        L.orc_char2rna.restype = C.c_int
        L.orc_bpla.restype = C.c_double
        L.orc_bpla.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double,
                               C.c_double, C.c_double, _D]
        L.orc_bpla_weights.argtypes = [C.c_void_p, _F, _F, _F]
        L.orc_stem4d.restype = C.c_double
        L.orc_stem4d.argtypes = [C.c_char_p, _D, C.c_char_p, _D, C.c_double, C.c_double,
                                 C.c_double, C.c_float, C.c_int, C.c_uint]
        L.orc_stem4d_ksum.restype = C.c_double
        L.orc_stem4d_ksum.argtypes = [C.c_char_p, _D, C.c_char_p, _D, C.c_double, C.c_double,
                                 C.c_double, C.c_float, C.c_int, C.c_uint]
        L.orc_stem4d_banded.restype = C.c_double
        L.orc_stem4d_banded.argtypes = [C.c_char_p, _D, C.c_char_p, _D, C.c_double, C.c_double,
                                        C.c_double, C.c_float, C.c_int, C.c_uint, C.c_uint]
        L.orc_stem4d_partial.restype = C.c_double
        L.orc_stem4d_partial.argtypes = [C.c_char_p, _D, C.c_char_p, _D, C.c_double, C.c_double,
                                         C.c_double, C.c_float, C.c_int, C.c_uint, C.c_uint,
                                         C.c_float, C.c_int]
        L.orc_phmm_posterior.restype = C.c_int
        L.orc_phmm_posterior.argtypes = [C.c_char_p, C.c_char_p, C.c_int, _D]
        L.orc_alignment_constraints.restype = C.c_int
        L.orc_alignment_constraints.argtypes = [C.c_char_p, C.c_char_p, C.c_float, C.c_uint,
                                                C.c_int, _U, _U]
        L.orc_bpla_gradients.restype = C.c_double
        L.orc_bpla_gradients.argtypes = [C.c_void_p, C.c_void_p, C.c_double, C.c_double,
                                         C.c_double, C.c_double, _D, _D]
        L.orc_naive_string.restype = C.c_double
        L.orc_naive_string.argtypes = [C.c_char_p, C.c_char_p, C.c_double]
        _o = L
    return _o


def reference_partial():
    """The reference's own rna.cpp/profile.cpp/ribosum.cpp (None if absent)."""
    global _r
    if _r is None:
        if not os.path.exists(REF_SO):
            return None
        L = C.CDLL(REF_SO)
        L.skref_char2rna.argtypes = [C.c_int]
        L.skref_char2rna.restype = C.c_int
        L.skref_profile.argtypes = [C.c_int, C.POINTER(C.c_char_p), _F, _F]
        L.skref_profile.restype = C.c_int
        L.skref_ribosum.argtypes = [_F, _F]
        _r = L
    return _r


class OMData:
    """Oracle MData (one example)."""

    def __init__(self, rows: Sequence[str], bpp_rows: Optional[Sequence[np.ndarray]], th=0.01,
                 use_bp=True):
        L = oracle()
        n = len(rows)
        self._rows = (C.c_char_p * n)(*[r.encode() for r in rows])
        self._keep = []
        barr = (_D * n)()
        if use_bp:
            for k, b in enumerate(bpp_rows):
                b = np.ascontiguousarray(b, dtype=np.float64)
                if b.size == 0:
                    b = np.zeros(1)
                self._keep.append(b)
                barr[k] = b.ctypes.data_as(_D)
        self.h = C.c_void_p(L.orc_mdata_new(n, self._rows, barr, C.c_float(th), int(use_bp)))

    def __del__(self):
        if getattr(self, "h", None) and _o is not None:
            _o.orc_mdata_free(self.h)
            self.h = None

    def dag(self) -> dict:
        L = oracle()
        nn = L.orc_mdata_n_nodes(self.h)
        ne = L.orc_mdata_n_edges(self.h)
        nb = L.orc_mdata_n_bpfreq(self.h)
        nr = L.orc_mdata_n_roots(self.h)
        sl = L.orc_mdata_seq_len(self.h)
        u = lambda k: np.zeros(max(k, 1), np.uint32)
        f = lambda k: np.zeros(max(k, 1), np.float32)
        first, last, ned, nbf, mp = u(nn), u(nn), u(nn), u(nn), u(nn)
        w = f(nn)
        L.orc_mdata_nodes(self.h, *(a.ctypes.data_as(_U) for a in (first, last, ned, nbf)),
                          w.ctypes.data_as(_F), mp.ctypes.data_as(_U))
        to, gaps = u(ne), u(ne)
        L.orc_mdata_edges(self.h, to.ctypes.data_as(_U), gaps.ctypes.data_as(_U))
        code, p = u(nb), f(nb)
        L.orc_mdata_bpfreq(self.h, code.ctypes.data_as(_U), p.ctypes.data_as(_F))
        roots = u(nr)
        L.orc_mdata_roots(self.h, roots.ctypes.data_as(_U))
        pw = f(sl)
        L.orc_mdata_weight(self.h, pw.ctypes.data_as(_F))
        return dict(first=first[:nn], last=last[:nn], n_edges=ned[:nn], n_bpfreq=nbf[:nn],
                    weight=w[:nn], max_pa=mp[:nn], edge_to=to[:ne], edge_gaps=gaps[:ne],
                    bp_code=code[:nb], bp_p=p[:nb], roots=roots[:nr], pos_weight=pw[:sl])


def su_stem(x: OMData, y: OMData, loop_gap=0.2, beta=0.3, band=10) -> float:
    return oracle().orc_su_stem(x.h, y.h, loop_gap, beta, band)


def si_stem(x: OMData, y: OMData, loop_gap=0.2, stack=1.3, covar=0.8, band=10) -> float:
    return oracle().orc_si_stem(x.h, y.h, loop_gap, stack, covar, band)


def su_str(x: OMData, y: OMData, gap=0.8, alpha=0.2) -> float:
    return oracle().orc_profile_string(x.h, y.h, gap, 1, alpha, 0.0, 0.0)


def si_str(x: OMData, y: OMData, gap=0.8, match=1.0, mismatch=0.8) -> float:
    return oracle().orc_profile_string(x.h, y.h, gap, 0, 0.0, match, mismatch)


def kernel_value(kind: int, x: OMData, y: OMData, p) -> float:
    """Composite kernels of def_kernel.h / conv_kernel.h from the components;
    p is a KernelParams-like object (attribute access)."""
    import math
    stem = lambda: su_stem(x, y, p.loop_gap, p.beta, p.len_band)
    if kind == 0:
        return stem()
    if kind == 1:
        return si_stem(x, y, p.loop_gap, p.stack, p.covar, p.len_band)
    if kind == 2:
        return su_str(x, y, p.gap, p.alpha)
    if kind == 3:
        return si_str(x, y, p.gap, p.match, p.mismatch)
    if kind == 4:
        return stem() + su_str(x, y, p.gap, p.alpha)
    if kind == 5:
        return si_stem(x, y, p.loop_gap, p.stack, p.covar, p.len_band) + si_str(x, y, p.gap, p.match, p.mismatch)
    if kind == 6:
        return p.beta * math.log(stem()) + 0.0
    if 9 <= kind <= 12:
        return bpla(x, y, kind in (10, 12), kind in (11, 12), p.gap, p.ext, p.alpha, p.beta,
                    list(p.score_table))
    if kind == 8:
        raise ValueError("naive string kernel compares raw strings: use naive_string()")
    if kind == 7:
        return (p.beta * math.log(stem()) + 0.0) + (p.alpha * math.log(su_str(x, y, p.gap, p.alpha)) + 0.0)
    raise ValueError(kind)


def naive_string(x: str, y: str, gap=0.8) -> float:
    return oracle().orc_naive_string(x.encode(), y.encode(), gap)


def bpla(x: OMData, y: OMData, no_bp: bool, sw: bool, gap, ext, alpha, beta, table16) -> float:
    t = (C.c_double * 16)(*table16)
    return oracle().orc_bpla(x.h, y.h, int(no_bp), int(sw), gap, ext, alpha, beta, t)


def bpla_weights(x: OMData):
    L = oracle().orc_mdata_seq_len(x.h)
    a = [np.zeros(max(L, 1), np.float32) for _ in range(3)]
    oracle().orc_bpla_weights(x.h, *(v.ctypes.data_as(_F) for v in a))
    return [v[:L] for v in a]


def stem4d(x: str, bpx, y: str, bpy, gap=0.8, stack=1.0, subst=0.5, bp_bound=0.0, model=0,
           loop=3, band=0, ali_bound=0.0, zerop_fixed=0) -> float:
    """StemKernel::operator() of stem_kernel/stem_kernel.h:52-55: full_dp
    (stem_kernel.cpp:282-351), or partial_dp (:113-280) when band or
    ali_bound is set (x, y as the loader gives them: lowercase)."""
    def arr(b):
        if b is None:
            return None
        b = np.ascontiguousarray(b, dtype=np.float64)
        return b.ctypes.data_as(_D) if b.size else np.zeros(1).ctypes.data_as(_D)
    keep = [np.ascontiguousarray(b, dtype=np.float64) if b is not None else None for b in (bpx, bpy)]
    px = keep[0].ctypes.data_as(_D) if keep[0] is not None and keep[0].size else None
    py = keep[1].ctypes.data_as(_D) if keep[1] is not None and keep[1].size else None
    if ali_bound > 0.0:
        return oracle().orc_stem4d_partial(x.encode(), px, y.encode(), py, gap, stack, subst,
                                           bp_bound, model, loop, band, ali_bound, zerop_fixed)
    if band:
        return oracle().orc_stem4d_banded(x.encode(), px, y.encode(), py, gap, stack, subst,
                                          bp_bound, model, loop, band)
    return oracle().orc_stem4d(x.encode(), px, y.encode(), py, gap, stack, subst, bp_bound,
                               model, loop)


def stem4d_ksum(x: str, bpx, y: str, bpy, gap=0.8, stack=1.0, subst=0.5, bp_bound=0.0, model=0,
                loop=3) -> float:
    """full_dp's K as 1 + the sum of the stacking sources (the engine's K-sum
    formulation), from the same loops as stem4d()."""
    keep = [np.ascontiguousarray(b, dtype=np.float64) if b is not None else None for b in (bpx, bpy)]
    px = keep[0].ctypes.data_as(_D) if keep[0] is not None and keep[0].size else None
    py = keep[1].ctypes.data_as(_D) if keep[1] is not None and keep[1].size else None
    return oracle().orc_stem4d_ksum(x.encode(), px, y.encode(), py, gap, stack, subst, bp_bound,
                                    model, loop)


def phmm_posterior(x: str, y: str, zerop_fixed=0) -> np.ndarray:
    """PairHMM posteriors fb[s, i, j] (stem_kernel/phmm.cpp:10-115)."""
    fb = np.zeros((3, len(x) + 1, len(y) + 1))
    if oracle().orc_phmm_posterior(x.encode(), y.encode(), zerop_fixed, fb.ctypes.data_as(_D)):
        raise ValueError("unknown nucleotide")
    return fb


def alignment_constraints(x: str, y: str, ali_bound: float, band=0, zerop_fixed=0):
    """StemKernel::alignment_constraints (stem_kernel/stem_kernel.cpp:14-81)."""
    lo = np.zeros(len(x) + 1, np.uint32)
    hi = np.zeros(len(x) + 1, np.uint32)
    if oracle().orc_alignment_constraints(x.encode(), y.encode(), ali_bound, band, zerop_fixed,
                                          lo.ctypes.data_as(_U), hi.ctypes.data_as(_U)):
        raise ValueError("unknown nucleotide")
    return lo, hi


def bpla_gradients(x: OMData, y: OMData, alpha, beta, gap, ext, table16):
    """BPLAKernel::compute_gradients (bpla_kernel.cpp:385-401): (value,
    [d_alpha, d_beta, d_gap, d_ext], backward total)."""
    t = np.ascontiguousarray(table16, dtype=np.float64)
    d = np.zeros(5)
    v = oracle().orc_bpla_gradients(x.h, y.h, alpha, beta, gap, ext, t.ctypes.data_as(_D),
                                    d.ctypes.data_as(_D))
    return v, d[:4].copy(), float(d[4])


# ------------------------------------------------------------------ McCaskill fold
def _fold_lib():
    L = oracle()
    if not getattr(L, "_fold_bound", False):
        L.orc_fold_mccaskill.restype = C.c_double
        L.orc_fold_mccaskill.argtypes = [C.c_char_p, C.c_int, C.c_int, _D]
        L.orc_fold_enum.restype = C.c_double
        L.orc_fold_enum.argtypes = [C.c_char_p, C.c_int, C.c_int, _D, C.POINTER(C.c_long)]
        L.orc_fold_structure_energy.restype = C.c_double
        L.orc_fold_structure_energy.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.c_int, C.c_int]
        L._fold_bound = True
    return L


def _fl(no_closing_gu, no_lp):
    """fold_oracle.c's third argument: bit 0 --noClosingGU, bit 1 --noLonelyPairs."""
    return int(bool(no_closing_gu)) | (2 if no_lp else 0)


def fold_mccaskill(seq: str, no_gu=False, no_closing_gu=False, no_lp=False):
    """(ln Z, packed bpp) of the restated McCaskill DP (fold_oracle.c)."""
    n = len(seq)
    bpp = np.zeros(max(n * (n - 1) // 2, 1))
    lz = _fold_lib().orc_fold_mccaskill(seq.encode(), int(no_gu), _fl(no_closing_gu, no_lp),
                                        bpp.ctypes.data_as(_D))
    return lz, bpp[: n * (n - 1) // 2]


def fold_enum(seq: str, no_gu=False, no_closing_gu=False, no_lp=False):
    """(ln Z, packed bpp, number of structures) by exhaustive enumeration."""
    n = len(seq)
    bpp = np.zeros(max(n * (n - 1) // 2, 1))
    cnt = C.c_long()
    lz = _fold_lib().orc_fold_enum(seq.encode(), int(no_gu), _fl(no_closing_gu, no_lp),
                                   bpp.ctypes.data_as(_D), C.byref(cnt))
    return lz, bpp[: n * (n - 1) // 2], cnt.value


def fold_structure_energy(seq: str, dotbracket: str, no_gu=False, no_closing_gu=False) -> float:
    st, pt = [], np.full(len(seq), -1, np.int32)
    for k, c in enumerate(dotbracket):
        if c == "(":
            st.append(k)
        elif c == ")":
            i = st.pop()
            pt[i], pt[k] = k, i
    return _fold_lib().orc_fold_structure_energy(seq.encode(), pt.ctypes.data_as(C.POINTER(C.c_int)),
                                                 int(no_gu), int(no_closing_gu))
