"""Host-side mirror of the reference's plugin interface for the hot path.

Names, argument meaning and defaults follow the reference:

* kernel classes -- ``stem_kernel_lite/def_kernel.h`` (SuStemKernel,
  SiStemKernel, SuStemStrKernel, SiStemStrKernel, LSuStemKernel,
  LSuStemStrKernel), ``stem_kernel_lite/string_kernel.h`` (StringKernel) and
  ``stem_kernel_lite/ss_kernel.h`` (StemStrKernel == SuStemStrKernel);
* ``Dataset`` -- the ExampleSet of (label, MData) that ``App::load_examples``
  builds (``common/framework.h:308-353``; ``MData`` ctor
  ``stem_kernel_lite/data.cpp:324-345``);
* ``KernelMatrix`` -- ``common/kernel_matrix.h:13-108``: ``calculate`` (train
  Gram / test x train), ``calculate_row`` (test row), ``diagonal``, ``print``.

Every computation goes through the HIP engine (libstem_kernel_amd.so); there
is no CPU fallback.  Errors raise ``StemKernelError`` (the reference threw
``const char*``).
"""
from __future__ import annotations

import ctypes as C
import sys
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import SK_OK, KernelParams, StemKernelError, check, lib

__all__ = [
    "fold", "random_sequences", "Dataset", "Context", "KernelMatrix",
    "SuStemKernel", "SiStemKernel", "StringKernel", "SuStemStrKernel", "StemStrKernel",
    "SiStemStrKernel", "LSuStemKernel", "LSuStemStrKernel", "NaiveStringKernel",
    "StemKernelError", "SVMModel",
]


# --------------------------------------------------------------------- inputs
_FORMATS = {"fa": _lib.FMT_FASTA, "fasta": _lib.FMT_FASTA, "aln": _lib.FMT_CLUSTAL,
            "clustal": _lib.FMT_CLUSTAL, "maf": _lib.FMT_MAF}


def _seqfile_rows(h) -> List[List[str]]:
    L = lib()
    try:
        return [[L.sk_seqfile_row(h, i, r).decode() for r in range(L.sk_seqfile_rows(h, i))]
                for i in range(L.sk_seqfile_count(h))]
    finally:
        L.sk_seqfile_free(h)


def _seqfile_check(rc):
    if rc != SK_OK:
        m = lib().sk_seqfile_last_error()
        raise StemKernelError(rc, m.decode() if m else "")


def read_examples(path: str, fmt: str = "fa") -> List[List[str]]:
    """Examples of a FASTA ("fa": one sequence each), CLUSTAL ("aln") or MAF
    ("maf") file, each a list of rows as written (load_fa / load_aln /
    load_maf, common/{fa,aln,maf}.cpp, through sk_seqfile_read)."""
    h = C.c_void_p()
    _seqfile_check(lib().sk_seqfile_read(path.encode(), _FORMATS[fmt], C.byref(h)))
    return _seqfile_rows(h)


def parse_examples(text: str, fmt: str = "fa") -> List[List[str]]:
    """read_examples over an in-memory text (sk_seqfile_parse)."""
    b = text.encode()
    h = C.c_void_p()
    _seqfile_check(lib().sk_seqfile_parse(b, len(b), _FORMATS[fmt], C.byref(h)))
    return _seqfile_rows(h)


def fold(seq: str, no_gu: bool = False) -> np.ndarray:
    """Synthetic base-pairing probabilities (Nussinov-Boltzmann stand-in for
    Vienna pf_fold), packed strict upper triangle of length n(n-1)/2."""
    n = len(seq)
    out = np.zeros(max(n * (n - 1) // 2, 1), dtype=np.float64)
    check(lib().sk_fold_synthetic(seq.encode(), n, int(no_gu),
                                  out.ctypes.data_as(C.POINTER(C.c_double))))
    return out[: n * (n - 1) // 2]


def random_sequences(n: int, length: int, seed: int) -> List[str]:
    """splitmix64 ACGU sequences (SURVEY.md §8d generator)."""
    st = C.c_uint64(seed)
    buf = C.create_string_buffer(n * (length + 1))
    check(lib().sk_random_sequences(C.byref(st), n, length, buf))
    raw = buf.raw
    return [raw[i * (length + 1): i * (length + 1) + length].decode() for i in range(n)]


# --------------------------------------------------------------------- kernels
class _Kernel:
    kind = _lib.SU_STEM

    def __init__(self, **kw):
        self.params = _lib.default_params(self.kind, **kw)

    def __repr__(self):
        p = self.params
        f = {k: getattr(p, k) for k, _ in KernelParams._fields_}
        return f"{type(self).__name__}({f})"


class SuStemKernel(_Kernel):
    """SuStemKernel(loop_gap, beta, len_band)  def_kernel.h:35-57 (--no-string)."""
    kind = _lib.SU_STEM

    def __init__(self, loop_gap=0.2, beta=0.3, len_band=10):
        super().__init__(loop_gap=loop_gap, beta=beta, len_band=len_band)


class SiStemKernel(_Kernel):
    """SiStemKernel(loop_gap, stack, covar, len_band)  def_kernel.h:11-33."""
    kind = _lib.SI_STEM

    def __init__(self, loop_gap=0.2, stack=1.3, covar=0.8, len_band=10):
        super().__init__(loop_gap=loop_gap, stack=stack, covar=covar, len_band=len_band)


class StringKernel(_Kernel):
    """StringKernel(gap, alpha) or StringKernel(gap, match, mismatch)
    (stem_kernel_lite/string_kernel.cpp:46-70)."""

    def __init__(self, gap=0.8, alpha=None, match=None, mismatch=None):
        if match is not None or mismatch is not None:
            self.kind = _lib.SI_STR
            super().__init__(gap=gap, match=1.0 if match is None else match,
                             mismatch=0.8 if mismatch is None else mismatch)
        else:
            self.kind = _lib.SU_STR
            super().__init__(gap=gap, alpha=0.2 if alpha is None else alpha)


class SuStemStrKernel(_Kernel):
    """SuStemStrKernel(alpha, beta, loop_gap, gap, len_band)  def_kernel.h:86-111;
    identical to StemStrKernel<SubstScoreTable> of ss_kernel.h:9-38."""
    kind = _lib.SU_STEM_STR

    def __init__(self, alpha=0.2, beta=0.3, loop_gap=0.2, gap=0.8, len_band=10):
        super().__init__(alpha=alpha, beta=beta, loop_gap=loop_gap, gap=gap, len_band=len_band)


StemStrKernel = SuStemStrKernel


class NaiveStringKernel(_Kernel):
    """StringKernel<double>(gap) of string_kernel/ (string_kernel.cpp:11-50):
    exact character match of the first row, weight gap^2, no profiles."""
    kind = _lib.NAIVE_STR

    def __init__(self, gap=0.8):
        super().__init__(gap=gap)


class BPLAKernel(_Kernel):
    """BPLAKernel<double,MData>(score_table, noBP, SW, gap, ext, alpha, beta)
    bpla_kernel/bpla_kernel.h:14-44, operator() bpla_kernel.cpp:159-174.

    noBP: LAScore only (no base-pairing terms); SW: Smith-Waterman maximum
    instead of the local-alignment partition function.  The reference CLI
    reads gap/ext/alpha/beta as float (bpla_kernel/main.cpp:52-76), so they
    are rounded to float32 here, as the CLI would; score_table (4x4, ACGU,
    x residue major) defaults to bpla_kernel/main.cpp:20-26."""

    def __init__(self, noBP=False, SW=False, gap=-8.0, ext=-0.75, alpha=4.5, beta=0.11,
                 score_table=None, cli_float=True):
        self.kind = {(False, False): _lib.BPLA, (True, False): _lib.LA,
                     (False, True): _lib.BPLA_SW, (True, True): _lib.LA_SW}[(bool(noBP), bool(SW))]
        f = (lambda v: float(np.float32(v))) if cli_float else float
        kw = dict(gap=f(gap), ext=f(ext), alpha=f(alpha), beta=f(beta))
        if score_table is not None:
            kw["score_table"] = np.asarray(score_table, dtype=np.float64).reshape(16)
        super().__init__(**kw)


class StemKernel4D(_Kernel):
    """StemKernel<double,BPMat>(use_GU, loop, gap, stack, subst, band,
    ali_bound, bp_bound) of stem_kernel/ (stem_kernel.h:26-60), full_dp
    (stem_kernel.cpp:282-351) over single sequences.

    bp_model 0 is the CLI's default -p path (BPMatrix: the dataset's base-pair
    probabilities, pairs counted when p > bp_bound); 1/2 are NormalBasePair /
    WobbleBasePair (-w), which the CLI runs with bp_bound 1.0 (so K = 1).
    Options are float on the CLI (stem_kernel/main.cpp:40-60) and are rounded
    to float32 here like the CLI would."""
    kind = _lib.STEM4D

    def __init__(self, gap=0.8, stack=1.0, subst=0.5, bp_bound=0.0, bp_model=0, loop=3, band=0,
                 ali_bound=0.0, ali_zerop_fixed=False, cli_float=True):
        """band > 0 or ali_bound > 0 selects partial_dp (stem_kernel.h:52-55)
        with the constraints of alignment_constraints (stem_kernel.cpp:14-81):
        -b band around the diagonal, -a anchors from the PairHMM MAP path
        (computed on the GPU).  ali_zerop_fixed picks LogValue's zerop
        semantics (see include/stem_kernel.h); both 0 is full_dp."""
        f = (lambda v: float(np.float32(v))) if cli_float else float
        super().__init__(gap=f(gap), stack=f(stack), subst=f(subst), bp_bound=f(bp_bound),
                         bp_model=int(bp_model), loop=int(loop), len_band=int(band),
                         ali_bound=float(np.float32(ali_bound)),
                         ali_zerop_fixed=int(bool(ali_zerop_fixed)))


class SiStemStrKernel(_Kernel):
    """SiStemStrKernel(loop_gap, stack, covar, gap, match, mismatch, len_band)
    def_kernel.h:58-84 (--no-ribosum)."""
    kind = _lib.SI_STEM_STR

    def __init__(self, loop_gap=0.2, stack=1.3, covar=0.8, gap=0.8, match=1.0, mismatch=0.8,
                 len_band=10):
        super().__init__(loop_gap=loop_gap, stack=stack, covar=covar, gap=gap, match=match,
                         mismatch=mismatch, len_band=len_band)


class LSuStemKernel(_Kernel):
    """LSuStemKernel: beta*log(K_stem)  def_kernel.h:113-138 (--log --no-string)."""
    kind = _lib.LSU_STEM

    def __init__(self, loop_gap=0.2, beta=0.3, len_band=10):
        super().__init__(loop_gap=loop_gap, beta=beta, len_band=len_band)


class LSuStemStrKernel(_Kernel):
    """LSuStemStrKernel: beta*log K_stem + alpha*log K_str  def_kernel.h:165-190 (--log)."""
    kind = _lib.LSU_STEM_STR

    def __init__(self, alpha=0.2, beta=0.3, loop_gap=0.2, gap=0.8, len_band=10):
        super().__init__(alpha=alpha, beta=beta, loop_gap=loop_gap, gap=gap, len_band=len_band)


# --------------------------------------------------------------------- data
class Dataset:
    """ExampleSet of (label, MData); examples are built on the host by the
    engine's DAG builder and uploaded once per device."""

    def __init__(self):
        self._h = C.c_void_p()
        check(lib().sk_dataset_create(C.byref(self._h)))
        self._uploaded_ctx = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.sk_dataset_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def add(self, label: str, rows: Sequence[str], bpp_rows: Optional[Sequence[np.ndarray]] = None,
            th: float = 0.01, use_bp: bool = True) -> None:
        """Append one example (an alignment of ``rows``).  ``bpp_rows[r]`` is the
        packed bp matrix of the gap-erased row r; computed with ``fold`` when
        omitted."""
        rows = list(rows)
        if use_bp and bpp_rows is None:
            bpp_rows = [fold(r.replace("-", "").lower()) for r in rows]
        n = len(rows)
        carr = (C.c_char_p * n)(*[r.encode() for r in rows])
        keep = []
        if use_bp:
            barr = (C.POINTER(C.c_double) * n)()
            for k, b in enumerate(bpp_rows):
                b = np.ascontiguousarray(b, dtype=np.float64)
                if b.size == 0:
                    b = np.zeros(1)
                keep.append(b)
                barr[k] = b.ctypes.data_as(C.POINTER(C.c_double))
        else:
            barr = None
        rc = lib().sk_dataset_add(self._h, label.encode(), n, carr, barr, C.c_float(th), int(use_bp))
        check(rc)

    def add_file(self, label: str, path: str, fmt: str = "fa", th: float = 0.01,
                 use_bp: bool = True) -> int:
        """Append every example of an example file, as DataLoader<MData>
        (stem_kernel_lite/data.cpp:456-586) does for one `label file` pair of
        the CLI; each row's bpp from ``fold`` (the synthetic stand-in for
        Vienna).  Returns the number of examples added."""
        alns = read_examples(path, fmt)
        for rows in alns:
            self.add(label, rows, th=th, use_bp=use_bp)
        return len(alns)

    @classmethod
    def from_sequences(cls, seqs: Iterable[str], labels: Optional[Iterable[str]] = None,
                       th: float = 0.01, bpp: Optional[Sequence[np.ndarray]] = None):
        ds = cls()
        seqs = list(seqs)
        labels = list(labels) if labels is not None else ["+1"] * len(seqs)
        for k, s in enumerate(seqs):
            ds.add(labels[k], [s], None if bpp is None else [bpp[k]], th=th)
        return ds

    @classmethod
    def synthetic(cls, seqs: Sequence[str], labels: Optional[Sequence[str]] = None,
                  th: float = 0.01, threads: int = 0):
        """Fold (synthetic model) and build all examples on host threads."""
        ds = cls()
        n = len(seqs)
        sarr = (C.c_char_p * n)(*[s.encode() for s in seqs])
        larr = None if labels is None else (C.c_char_p * n)(*[l.encode() for l in labels])
        check(lib().sk_dataset_add_synthetic(ds._h, n, sarr, larr, C.c_float(th), threads))
        return ds

    @classmethod
    def synthetic_alignments(cls, alns: Sequence[Sequence[str]], labels=None, th: float = 0.01,
                             threads: int = 0):
        """Alignments with the same row count: fold every row on host threads."""
        ds = cls()
        n = len(alns)
        nr = len(alns[0]) if n else 1
        if any(len(a) != nr for a in alns):
            raise ValueError("synthetic_alignments needs the same number of rows per alignment")
        flat = [r.encode() for a in alns for r in a]
        rarr = (C.c_char_p * max(len(flat), 1))(*flat)
        larr = None if labels is None else (C.c_char_p * n)(*[l.encode() for l in labels])
        check(lib().sk_dataset_add_synthetic_rows(ds._h, n, nr, rarr, larr, C.c_float(th),
                                                  threads))
        return ds

    def add_batch(self, alns: Sequence[Sequence[str]], bpp_rows=None, labels=None,
                  th: float = 0.01, use_bp: bool = True, threads: int = 0) -> None:
        """Append alignments of equal row count, built on host threads from
        the caller's per-row bpp (``bpp_rows[i][r]``, packed, of the
        gap-erased row; sk_dataset_add_batch)."""
        n = len(alns)
        nr = len(alns[0]) if n else 1
        if any(len(a) != nr for a in alns):
            raise ValueError("add_batch needs the same number of rows per alignment")
        flat = [r.encode() for a in alns for r in a]
        rarr = (C.c_char_p * max(len(flat), 1))(*flat)
        larr = None if labels is None else (C.c_char_p * n)(*[l.encode() for l in labels])
        keep, barr = [], None
        if use_bp:
            barr = (C.POINTER(C.c_double) * max(n * nr, 1))()
            for i in range(n):
                for r in range(nr):
                    b = np.ascontiguousarray(bpp_rows[i][r], dtype=np.float64)
                    if b.size == 0:
                        b = np.zeros(1)
                    keep.append(b)
                    barr[i * nr + r] = b.ctypes.data_as(C.POINTER(C.c_double))
        check(lib().sk_dataset_add_batch(self._h, n, nr, rarr, barr, larr, C.c_float(th),
                                         int(use_bp), threads))

    @classmethod
    def folded(cls, ctx: "Context", alns, labels=None, th: float = 0.01, no_gu: bool = False,
               no_closing_gu: bool = False, threads: int = 0, no_lonely_pairs: bool = False):
        """Examples whose rows are folded on ctx's GPU (sk_fold_mccaskill, the
        engine's McCaskill in place of Vienna pf_fold) and built on host
        threads (sk_dataset_add_folded).  ``alns``: sequences or alignments
        of equal row count."""
        alns = [[a] if isinstance(a, str) else list(a) for a in alns]
        ds = cls()
        n = len(alns)
        nr = len(alns[0]) if n else 1
        if any(len(a) != nr for a in alns):
            raise ValueError("folded needs the same number of rows per alignment")
        flat = [r.encode() for a in alns for r in a]
        rarr = (C.c_char_p * max(len(flat), 1))(*flat)
        larr = None if labels is None else (C.c_char_p * n)(*[l.encode() for l in labels])
        flags = (1 if no_gu else 0) | (2 if no_closing_gu else 0) | (4 if no_lonely_pairs else 0)
        ctx._chk(lib().sk_dataset_add_folded(ctx.handle, ds._h, n, nr, rarr, larr, C.c_float(th),
                                             flags, threads))
        return ds

    def __len__(self):
        return lib().sk_dataset_size(self._h)

    def export(self, first: int = 0, count: Optional[int] = None) -> bytearray:
        """Examples [first, first + count) as bytes (sk_dataset_export): their
        labels and built DAGs, profiles, weights and bp matrices."""
        count = len(self) - first if count is None else count
        need = C.c_size_t()
        check(lib().sk_dataset_export(self._h, first, count, None, 0, C.byref(need)))
        out = bytearray(need.value)  # written in place (no intermediate copy)
        buf = (C.c_char * max(need.value, 1)).from_buffer(out) if need.value else None
        check(lib().sk_dataset_export(self._h, first, count, buf, need.value, C.byref(need)))
        return out

    def import_bytes(self, data) -> "Dataset":
        """Append the examples of an export() (sk_dataset_import; bytes or
        bytearray)."""
        n = len(data)
        if isinstance(data, bytearray) and n:
            data = (C.c_char * n).from_buffer(data)
        check(lib().sk_dataset_import(self._h, data, n))
        return self

    def pack_digest(self):
        """(y-role, x-role) hashes of the host-packed arrays
        (sk_dataset_pack_digest; the dataset must not be uploaded)."""
        hy, hx = C.c_uint64(), C.c_uint64()
        check(lib().sk_dataset_pack_digest(self._h, C.byref(hy), C.byref(hx)))
        return hy.value, hx.value

    def profile(self, i: int):
        """ProfileSequence columns [len][5] and n_seqs of example i."""
        L = self.shape(i)[4]
        out = np.zeros((max(L, 1), 5), np.float32)
        ns = C.c_float()
        check(lib().sk_dataset_profile(self._h, i, out.ctypes.data_as(C.POINTER(C.c_float)),
                                       C.byref(ns)))
        return out[:L], ns.value

    def bpla_weights(self, i: int):
        """sqrt p_left, p_right, p_unpair of example i (bpla_kernel/data.cpp:19-45)."""
        L = self.shape(i)[4]
        a = [np.zeros(max(L, 1), np.float32) for _ in range(3)]
        check(lib().sk_dataset_bpla_weights(self._h, i, *(v.ctypes.data_as(C.POINTER(C.c_float))
                                                           for v in a)))
        return [v[:L] for v in a]

    def label(self, i: int) -> str:
        return lib().sk_dataset_label(self._h, i).decode()

    def shape(self, i: int):
        v = [C.c_int32() for _ in range(5)]
        check(lib().sk_dataset_shape(self._h, i, *[C.byref(a) for a in v]))
        return tuple(a.value for a in v)  # nodes, edges, bpfreq, roots, len

    def row_traffic(self, i: int) -> dict:
        """Row transfers of example i in the DAG stem kernel's gamma schedule
        (sk_dataset_row_traffic; the dataset must be uploaded)."""
        v = [C.c_int32() for _ in range(7)]
        check(lib().sk_dataset_row_traffic(self._h, i, *[C.byref(a) for a in v]))
        return dict(zip(("rows", "stored", "slab_reads", "gamma_reads", "phi_reads", "reg_reads",
                         "y_slots"), (a.value for a in v)))

    def dag(self, i: int) -> dict:
        """The DAG of example i (reference numbering), for packer parity."""
        nn, ne, nb, nr, L = self.shape(i)
        u = lambda k: np.zeros(max(k, 1), np.uint32)
        f = lambda k: np.zeros(max(k, 1), np.float32)
        d = dict(first=u(nn), last=u(nn), n_edges=u(nn), n_bpfreq=u(nn), weight=f(nn),
                 max_pa=u(nn), edge_to=u(ne), edge_gaps=u(ne), bp_code=u(nb), bp_p=f(nb),
                 roots=u(nr), pos_weight=f(L))
        ptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32 if a.dtype == np.uint32 else C.c_float))
        check(lib().sk_dataset_dag(self._h, i, *[ptr(d[k]) for k in
                                                 ("first", "last", "n_edges", "n_bpfreq", "weight",
                                                  "max_pa", "edge_to", "edge_gaps", "bp_code",
                                                  "bp_p", "roots", "pos_weight")]))
        sizes = dict(first=nn, last=nn, n_edges=nn, n_bpfreq=nn, weight=nn, max_pa=nn,
                     edge_to=ne, edge_gaps=ne, bp_code=nb, bp_p=nb, roots=nr, pos_weight=L)
        return {k: v[: sizes[k]] for k, v in d.items()}


# --------------------------------------------------------------------- device
class Context:
    """One context per GPU (sk_open)."""

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        self._h = C.c_void_p()
        check(lib().sk_open(device, C.c_void_p(stream) if stream else None, C.byref(self._h)))
        self.device = device

    def close(self):
        if self._h is not None and self._h.value:
            lib().sk_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def _chk(self, rc):
        return check(rc, self._h)

    def fold(self, seqs: Sequence[str], no_gu: bool = False, no_closing_gu: bool = False,
             log_z: bool = False, no_lonely_pairs: bool = False):
        """McCaskill base-pairing probabilities of every sequence on this GPU
        (sk_fold_mccaskill): a list of packed upper triangles, plus ln Z per
        sequence when ``log_z``."""
        seqs = list(seqs)
        n = len(seqs)
        sizes = [len(s) * (len(s) - 1) // 2 for s in seqs]
        out = np.zeros(max(sum(sizes), 1))
        lz = np.zeros(max(n, 1))
        sarr = (C.c_char_p * max(n, 1))(*[s.encode() for s in seqs])
        flags = (1 if no_gu else 0) | (2 if no_closing_gu else 0) | (4 if no_lonely_pairs else 0)
        self._chk(lib().sk_fold_mccaskill(self._h, n, sarr, flags,
                                          out.ctypes.data_as(C.POINTER(C.c_double)),
                                          lz.ctypes.data_as(C.POINTER(C.c_double))))
        res, o = [], 0
        for z in sizes:
            res.append(out[o:o + z].copy())
            o += z
        return (res, lz[:n]) if log_z else res

    def upload(self, ds: Dataset):
        self._chk(lib().sk_dataset_upload(self._h, ds.handle))

    def gram(self, ds: Dataset, kernel: _Kernel, normalize: bool = False) -> np.ndarray:
        self.upload(ds)
        n = len(ds)
        out = np.zeros((n, n), dtype=np.float64)
        self._chk(lib().sk_gram(self._h, ds.handle, C.byref(kernel.params), int(normalize),
                                out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def pairs(self, ds: Dataset, kernel: _Kernel, x, y) -> np.ndarray:
        self.upload(ds)
        x = np.ascontiguousarray(x, dtype=np.int32)
        y = np.ascontiguousarray(y, dtype=np.int32)
        out = np.zeros(x.size, dtype=np.float64)
        self._chk(lib().sk_pairs(self._h, ds.handle, C.byref(kernel.params),
                                 x.ctypes.data_as(C.POINTER(C.c_int32)),
                                 y.ctypes.data_as(C.POINTER(C.c_int32)), x.size,
                                 out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def bpla_gradients(self, ds: Dataset, kernel: "BPLAKernel", x, y, ys: Optional[Dataset] = None):
        """BPLAKernel::compute_gradients for pairs (ds[x[k]], (ys or ds)[y[k]])
        (bpla_kernel.cpp:385-401, the bpla_optimizer's per-pair step): returns
        (values[n], grads[n, 4] = d/d(alpha, beta, gap, ext))."""
        ys = ds if ys is None else ys
        self.upload(ds)
        self.upload(ys)
        x = np.ascontiguousarray(x, dtype=np.int32)
        y = np.ascontiguousarray(y, dtype=np.int32)
        val = np.zeros(x.size, dtype=np.float64)
        grad = np.zeros((x.size, 4), dtype=np.float64)
        self._chk(lib().sk_bpla_gradients(self._h, ds.handle, ys.handle, C.byref(kernel.params),
                                          x.ctypes.data_as(C.POINTER(C.c_int32)),
                                          y.ctypes.data_as(C.POINTER(C.c_int32)), x.size,
                                          val.ctypes.data_as(C.POINTER(C.c_double)),
                                          grad.ctypes.data_as(C.POINTER(C.c_double))))
        return val, grad

    def bpla_gradient_gram(self, ds: Dataset, kernel: "BPLAKernel", normalize: bool = False):
        """The bpla_optimizer's Gram and gradient matrices: CalcMatrix
        (bpla_optimizer.cpp:52-126; K[i,j] and dK/d(alpha, beta, gap, ext) for
        i <= j, mirrored) or, with normalize, CalcMatrixN (:128-255;
        K/sqrt(K_ii K_jj) and its derivative, diagonal 1 and 0).  Returns
        (K[n, n], G[4, n, n]); one sk_bpla_gradients call over all pairs."""
        from .shard import assemble_gradients
        n = len(ds)
        iu, ju = np.triu_indices(n)
        val, grad = self.bpla_gradients(ds, kernel, iu, ju)
        return assemble_gradients(iu, ju, val, grad, n, normalize)

    def comm_init(self, uid: bytes, rank: int, world: int) -> None:
        """This context's RCCL communicator (sk_comm_init); uid = the 128
        bytes rank 0 drew with sk_comm_unique_id (see shard.rccl_init)."""
        self._chk(lib().sk_comm_init(self._h, uid, len(uid), rank, world))

    def allgather(self, send_ptr: int, count: int, recv_ptr: int) -> None:
        """ncclAllGather of `count` doubles per rank on the context's stream
        (sk_comm_allgather; device pointers)."""
        self._chk(lib().sk_comm_allgather(self._h, send_ptr, count, recv_ptr))

    def gram_sharded(self, ds: Dataset, kernel: _Kernel, normalize: bool = False) -> np.ndarray:
        """The Gram over this context's communicator (sk_gram_sharded): the
        reference MPI Gram's cyclic cell plan, one RCCL all-gather, the whole
        matrix on every rank (common/kernel_matrix.cpp:186-261, 495-527)."""
        self.upload(ds)
        n = len(ds)
        out = np.zeros((n, n), dtype=np.float64)
        self._chk(lib().sk_gram_sharded(self._h, ds.handle, C.byref(kernel.params),
                                        int(normalize), out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def pairs_device(self, ds: Dataset, kernel: _Kernel, x, y, out_ptr: int) -> None:
        self.upload(ds)
        x = np.ascontiguousarray(x, dtype=np.int32)
        y = np.ascontiguousarray(y, dtype=np.int32)
        self._chk(lib().sk_pairs_device(self._h, ds.handle, C.byref(kernel.params),
                                        x.ctypes.data_as(C.POINTER(C.c_int32)),
                                        y.ctypes.data_as(C.POINTER(C.c_int32)), x.size,
                                        C.c_void_p(out_ptr)))

    def test_row(self, test: Dataset, t: int, train: Dataset, kernel: _Kernel,
                 sv_index=None, self_value: bool = False):
        self.upload(test)
        self.upload(train)
        out = np.zeros(len(train), dtype=np.float64)
        sv = None if sv_index is None else np.ascontiguousarray(sv_index, dtype=np.int32)
        sf = C.c_double(0.0)
        self._chk(lib().sk_test_row(self._h, test.handle, t, train.handle,
                                    None if sv is None else sv.ctypes.data_as(C.POINTER(C.c_int32)),
                                    0 if sv is None else sv.size, C.byref(kernel.params),
                                    out.ctypes.data_as(C.POINTER(C.c_double)),
                                    C.byref(sf) if self_value else None))
        return (out, sf.value) if self_value else out

    def diagonal(self, ds: Dataset, kernel: _Kernel, sv_index=None) -> np.ndarray:
        self.upload(ds)
        out = np.zeros(len(ds), dtype=np.float64)
        sv = None if sv_index is None else np.ascontiguousarray(sv_index, dtype=np.int32)
        self._chk(lib().sk_diagonal(self._h, ds.handle,
                                    None if sv is None else sv.ctypes.data_as(C.POINTER(C.c_int32)),
                                    0 if sv is None else sv.size, C.byref(kernel.params),
                                    out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def test_matrix(self, test: Dataset, train: Dataset, kernel: _Kernel, norm_test=False,
                    normalize=False):
        self.upload(test)
        self.upload(train)
        out = np.zeros((len(test), len(train)), dtype=np.float64)
        self_ = np.zeros(len(test), dtype=np.float64)
        self._chk(lib().sk_test_matrix(self._h, test.handle, train.handle, C.byref(kernel.params),
                                       int(norm_test), int(normalize),
                                       out.ctypes.data_as(C.POINTER(C.c_double)),
                                       self_.ctypes.data_as(C.POINTER(C.c_double))))
        return out, self_

    def last_timing(self):
        a, b, c, d = C.c_double(), C.c_double(), C.c_double(), C.c_int32()
        self._chk(lib().sk_last_timing(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return dict(stem_ms=a.value, string_ms=b.value, cells=c.value, launches=d.value)

    def set_async(self, on: bool = True) -> None:
        """sk_set_async: compute calls return once enqueued (results on the
        device after a stream sync); timings then come from sync_timing()."""
        self._chk(lib().sk_set_async(self._h, 1 if on else 0))

    def sync_timing(self) -> None:
        """sk_sync_timing: wait for every asynchronous call since the last
        sync_timing; last_timing() / last_launch_ms() then report their sums."""
        self._chk(lib().sk_sync_timing(self._h))

    def last_launch_ms(self):
        """Per-launch HIP-event durations of the last call's dominant kernel:
        (summed ms, launch count); launches on several streams overlap."""
        a, b = C.c_double(), C.c_int32()
        self._chk(lib().sk_last_launch_ms(self._h, C.byref(a), C.byref(b)))
        return dict(ms_sum=a.value, launches=b.value)

    def last_classes(self):
        """Kernel instantiations the last compute call launched: the DAG stem
        register classes (MAXK values; 0 = the big-y kernel, dag_stem_big.hip)
        and the 4-D classes as (CPL, banded); `stem4d_col` lists the CPLs that
        ran the column-pipelined full_dp kernel (also in `stem4d`, unbanded)."""
        a, b = C.c_uint32(), C.c_uint32()
        self._chk(lib().sk_last_classes(self._h, C.byref(a), C.byref(b)))
        # bit MAXK / 4 for the classes of multiples of 4 (0: the big-y kernel),
        # bit 17 for the MAXK 17 class
        maxk = sorted((4 * k if k <= 8 else k) for k in range(32) if a.value >> k & 1)
        s4d = sorted({(1 << (k & 3), bool(k & 4)) for k in range(12) if b.value >> k & 1})
        col = sorted(1 << (k & 3) for k in range(8, 12) if b.value >> k & 1)
        return dict(stem_maxk=maxk, stem4d=s4d, stem4d_col=col)


def stem4d_col_shape(min_len: int, max_len: int) -> dict:
    """Shape of the column-pipelined 4-D kernel for a batch of y examples of
    lengths [min_len, max_len] (sk_stem4d_col_shape): chained columns per
    group, waves per pair and rows fetched ahead per wave."""
    v = [C.c_int32() for _ in range(3)]
    check(lib().sk_stem4d_col_shape(int(min_len), int(max_len), *[C.byref(a) for a in v]))
    return dict(nb=v[0].value, waves=v[1].value, pf=v[2].value)


def format_libsvm(matrix: np.ndarray, labels: Sequence[str]) -> str:
    m = np.ascontiguousarray(matrix, dtype=np.float64)
    rows, cols = m.shape
    larr = (C.c_char_p * rows)(*[l.encode() for l in labels])
    need = C.c_size_t()
    check(lib().sk_format_libsvm(m.ctypes.data_as(C.POINTER(C.c_double)), rows, cols, larr, None,
                                 0, C.byref(need)))
    buf = C.create_string_buffer(need.value)
    check(lib().sk_format_libsvm(m.ctypes.data_as(C.POINTER(C.c_double)), rows, cols, larr, buf,
                                 need.value, C.byref(need)))
    return buf.value.decode()


class SVMModel:
    """A libsvm model for predict mode's Output (f3): SVMPredict
    (libsvm/svm_util.cpp:11-95) over the reference's libsvm 2.8x
    (sk_svm_model_load / sk_svm_predict, csrc/host/svm_predict.cpp)."""

    def __init__(self, path: str):
        h = C.c_void_p()
        rc = lib().sk_svm_model_load(str(path).encode(), C.byref(h))
        if rc != SK_OK:
            raise StemKernelError(rc, lib().sk_svm_last_error().decode())
        self._h = h
        t, k, p = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().sk_svm_model_info(self._h, C.byref(t), C.byref(k), None, C.byref(p)))
        self.svm_type, self.nr_class, self.has_probability = t.value, k.value, bool(p.value)
        labels = (C.c_int32 * max(k.value, 1))()
        check(lib().sk_svm_model_info(self._h, None, None, labels, None))
        self.labels = [labels[i] for i in range(k.value)]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().sk_svm_model_free(h)
            self._h = None

    def predict(self, row, cnt: int = 1, probability: bool = True):
        """(label, values) of SVMPredict::do_svm_predict for the test row
        (kernel values against the training examples, in training order):
        class probabilities for C-SVC / nu-SVC with probability, else the
        one-vs-one decision values."""
        r = np.ascontiguousarray(row, dtype=np.float64)
        nv = max(self.nr_class * (self.nr_class - 1) // 2, self.nr_class, 1)
        vals = np.zeros(nv, dtype=np.float64)
        label = C.c_double()
        rc = lib().sk_svm_predict(self._h, int(cnt), r.ctypes.data_as(C.POINTER(C.c_double)), r.size,
                                  int(probability), C.byref(label), vals.ctypes.data_as(C.POINTER(C.c_double)))
        if rc != SK_OK:
            raise StemKernelError(rc, lib().sk_svm_last_error().decode())
        if probability and self.svm_type in (0, 1):
            return label.value, vals[: self.nr_class]
        return label.value, vals[: max(self.nr_class * (self.nr_class - 1) // 2, 1)]


class KernelMatrix:
    """Mirror of KernelMatrix<double> (common/kernel_matrix.h:13-108)."""

    def __init__(self, ctx: Optional[Context] = None):
        self.ctx = ctx if ctx is not None else Context(0)
        self.matrix = np.zeros((0, 0))
        self.self_ = np.zeros(0)
        self.label: List[str] = []

    def calculate(self, train: Dataset, kernel: _Kernel, normalize: bool = False, n_th: int = 1):
        """Train Gram (kernel_matrix.cpp:485-575).  n_th is accepted for API
        parity; the GPU decides its own parallelism."""
        self.matrix = self.ctx.gram(train, kernel, normalize)
        self.label = [train.label(i) for i in range(len(train))]
        return 0.0

    def calculate_test(self, test: Dataset, train: Dataset, kernel: _Kernel, norm_test=False,
                       normalize=False, n_th: int = 1):
        """Test x train (kernel_matrix.cpp:699-754)."""
        self.matrix, self.self_ = self.ctx.test_matrix(test, train, kernel, norm_test, normalize)
        self.label = [test.label(i) for i in range(len(test))]
        return 0.0

    @staticmethod
    def calculate_row(ctx: Context, data: Dataset, t: int, train: Dataset, kernel: _Kernel,
                      sv_index=None, want_self=False):
        """Test row (kernel_matrix.cpp:635-697)."""
        return ctx.test_row(data, t, train, kernel, sv_index, want_self)

    @staticmethod
    def diagonal(ctx: Context, train: Dataset, kernel: _Kernel, sv_index=None):
        """kernel_matrix.cpp:577-633."""
        return ctx.diagonal(train, kernel, sv_index)

    def __call__(self, i, j=None):
        return self.self_[i] if j is None else self.matrix[i, j]

    def print(self, out=sys.stdout):
        """libsvm precomputed-kernel layout (kernel_matrix.cpp:756-770)."""
        out.write(format_libsvm(self.matrix, self.label))

    def save(self, path: str) -> None:
        """App's output file (common/framework.h:138-160): the libsvm text,
        gzip-compressed when the name ends in ".gz" and bzip2 when ".bz2"."""
        text = format_libsvm(self.matrix, self.label).encode()
        if path.endswith(".gz"):
            import gzip
            with gzip.open(path, "wb") as f:
                f.write(text)
        elif path.endswith(".bz2"):
            import bz2
            with bz2.open(path, "wb") as f:
                f.write(text)
        else:
            try:
                with open(path, "wb") as f:
                    f.write(text)
            except OSError as e:
                raise StemKernelError(-1, f"{path}: cannot open for writing") from e
