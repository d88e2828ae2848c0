"""ctypes binding of the C ABI in include/stem_kernel.h.

The shared library is built in-tree (``make`` or ``__graft_entry__.build()``)
as ``stem_kernel_amd/libstem_kernel_amd.so``.  There is no fallback: if the
library is missing, ``lib()`` raises.

torch, when importable, is imported *before* the library is loaded so that
both resolve the same ``libamdhip64.so.7`` (one HIP runtime per process).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SK_LIB_PATH") or os.path.join(_HERE, "libstem_kernel_amd.so")

SK_OK = 0
STATUS = {
    0: "ok", -1: "invalid argument", -2: "HIP runtime error", -3: "no usable gfx950 device",
    -4: "allocation failed", -5: "index out of range", -6: "unsupported",
}

# sk_kernel_kind
FMT_FASTA, FMT_CLUSTAL, FMT_MAF = range(3)
(SU_STEM, SI_STEM, SU_STR, SI_STR, SU_STEM_STR, SI_STEM_STR, LSU_STEM, LSU_STEM_STR, NAIVE_STR,
 BPLA, LA, BPLA_SW, LA_SW, STEM4D) = range(14)


class KernelParams(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("len_band", C.c_uint32), ("beta", C.c_double),
        ("loop_gap", C.c_double), ("stack", C.c_double), ("covar", C.c_double),
        ("alpha", C.c_double), ("gap", C.c_double), ("match", C.c_double),
        ("mismatch", C.c_double), ("ext", C.c_double), ("score_table", C.c_double * 16),
        ("subst", C.c_double), ("bp_bound", C.c_double), ("bp_model", C.c_int32),
        ("loop", C.c_uint32), ("ali_bound", C.c_double), ("ali_zerop_fixed", C.c_int32),
    ]


_P = C.c_void_p
_I32P = C.POINTER(C.c_int32)
_U32P = C.POINTER(C.c_uint32)
_F32P = C.POINTER(C.c_float)
_F64P = C.POINTER(C.c_double)

# name -> (restype, argtypes); every symbol include/stem_kernel.h declares
SIGNATURES = {
    "sk_kernel_params_default": (None, [C.POINTER(KernelParams), C.c_int32]),
    "sk_open": (C.c_int, [C.c_int, _P, C.POINTER(_P)]),
    "sk_close": (C.c_int, [_P]),
    "sk_strerror": (C.c_char_p, [C.c_int]),
    "sk_last_error": (C.c_char_p, [_P]),
    "sk_dataset_create": (C.c_int, [C.POINTER(_P)]),
    "sk_dataset_free": (C.c_int, [_P]),
    "sk_dataset_add": (C.c_int, [_P, C.c_char_p, C.c_int, C.POINTER(C.c_char_p),
                                 C.POINTER(_F64P), C.c_float, C.c_int]),
    "sk_dataset_add_synthetic": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_char_p),
                                           C.POINTER(C.c_char_p), C.c_float, C.c_int32]),
    "sk_dataset_add_synthetic_rows": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_char_p),
                                                C.POINTER(C.c_char_p), C.c_float, C.c_int32]),
    "sk_dataset_size": (C.c_int, [_P]),
    "sk_dataset_add_copy": (C.c_int, [_P, _P, C.c_int32]),
    "sk_dataset_export": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_void_p, C.c_size_t,
                                    C.POINTER(C.c_size_t)]),
    "sk_dataset_import": (C.c_int, [_P, C.c_void_p, C.c_size_t]),
    "sk_dataset_pack_digest": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "sk_dataset_label": (C.c_char_p, [_P, C.c_int]),
    "sk_dataset_shape": (C.c_int, [_P, C.c_int, _I32P, _I32P, _I32P, _I32P, _I32P]),
    "sk_dataset_row_traffic": (C.c_int, [_P, C.c_int, _I32P, _I32P, _I32P, _I32P, _I32P, _I32P, _I32P]),
    "sk_dataset_dag": (C.c_int, [_P, C.c_int, _U32P, _U32P, _U32P, _U32P, _F32P, _U32P,
                                 _U32P, _U32P, _U32P, _F32P, _U32P, _F32P]),
    "sk_dataset_profile": (C.c_int, [_P, C.c_int, _F32P, _F32P]),
    "sk_dataset_bpla_weights": (C.c_int, [_P, C.c_int, _F32P, _F32P, _F32P]),
    "sk_dataset_upload": (C.c_int, [_P, _P]),
    "sk_gram": (C.c_int, [_P, _P, C.POINTER(KernelParams), C.c_int, _F64P]),
    "sk_pairs_device": (C.c_int, [_P, _P, C.POINTER(KernelParams), _I32P, _I32P, C.c_int64,
                                  C.c_void_p]),
    "sk_pairs": (C.c_int, [_P, _P, C.POINTER(KernelParams), _I32P, _I32P, C.c_int64, _F64P]),
    "sk_test_row": (C.c_int, [_P, _P, C.c_int, _P, _I32P, C.c_int32, C.POINTER(KernelParams),
                              _F64P, _F64P]),
    "sk_diagonal": (C.c_int, [_P, _P, _I32P, C.c_int32, C.POINTER(KernelParams), _F64P]),
    "sk_test_matrix": (C.c_int, [_P, _P, _P, C.POINTER(KernelParams), C.c_int, C.c_int, _F64P,
                                 _F64P]),
    "sk_format_libsvm": (C.c_int, [_F64P, C.c_int32, C.c_int32, C.POINTER(C.c_char_p),
                                   C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "sk_fold_synthetic": (C.c_int, [C.c_char_p, C.c_int32, C.c_int32, _F64P]),
    "sk_fold_mccaskill": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_char_p), C.c_int32, _F64P, _F64P]),
    "sk_dataset_add_batch": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_char_p),
                                       C.POINTER(_F64P), C.POINTER(C.c_char_p), C.c_float,
                                       C.c_int32, C.c_int32]),
    "sk_dataset_add_folded": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.POINTER(C.c_char_p),
                                        C.POINTER(C.c_char_p), C.c_float, C.c_int32, C.c_int32]),
    "sk_random_sequences": (C.c_int, [C.POINTER(C.c_uint64), C.c_int32, C.c_int32, C.c_char_p]),
    "sk_last_timing": (C.c_int, [_P, _F64P, _F64P, _F64P, _I32P]),
    "sk_last_launch_ms": (C.c_int, [_P, _F64P, _I32P]),
    "sk_set_async": (C.c_int, [_P, C.c_int32]),
    "sk_sync_timing": (C.c_int, [_P]),
    "sk_shard_count": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "sk_shard_cells": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, _I32P, _I32P]),
    "sk_shard_assemble": (C.c_int, [C.c_int32, C.c_int32, _F64P, C.c_int64, C.c_int, _F64P]),
    "sk_comm_unique_id": (C.c_int, [C.c_char_p, C.c_size_t]),
    "sk_comm_init": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_int32, C.c_int32]),
    "sk_comm_allgather": (C.c_int, [_P, C.c_void_p, C.c_int64, C.c_void_p]),
    "sk_gram_sharded": (C.c_int, [_P, _P, C.POINTER(KernelParams), C.c_int, _F64P]),
    "sk_last_classes": (C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "sk_stem4d_col_shape": (C.c_int, [C.c_int32, C.c_int32, _I32P, _I32P, _I32P]),
    "sk_ribosum_tables": (None, [_F32P, _F32P]),
    "sk_char2rna": (C.c_int, [C.c_int]),
    "sk_experiments": (C.c_int, []),
    "sk_bpla_gradients": (C.c_int, [_P, _P, _P, C.POINTER(KernelParams), _I32P, _I32P, C.c_int64,
                                    _F64P, _F64P]),
    "sk_seqfile_read": (C.c_int, [C.c_char_p, C.c_int32, C.POINTER(_P)]),
    "sk_seqfile_parse": (C.c_int, [C.c_char_p, C.c_size_t, C.c_int32, C.POINTER(_P)]),
    "sk_seqfile_free": (C.c_int, [_P]),
    "sk_seqfile_count": (C.c_int64, [_P]),
    "sk_seqfile_rows": (C.c_int32, [_P, C.c_int64]),
    "sk_seqfile_row": (C.c_char_p, [_P, C.c_int64, C.c_int32]),
    "sk_seqfile_last_error": (C.c_char_p, []),
    "sk_svm_model_load": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "sk_svm_model_free": (None, [_P]),
    "sk_svm_model_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                    C.POINTER(C.c_int32)]),
    "sk_svm_predict": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_double), C.c_int32, C.c_int32,
                                 C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "sk_svm_last_error": (C.c_char_p, []),
}

_lock = threading.Lock()
_lib = None


class StemKernelError(RuntimeError):
    """Raised for a negative sk_status (the reference threw ``const char*``)."""

    def __init__(self, code, msg=""):
        super().__init__(f"{STATUS.get(code, code)}{': ' + msg if msg else ''}")
        self.code = code


def lib():
    """Load libstem_kernel_amd.so (raises if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise StemKernelError(-3, f"{LIB_PATH} not built; run `make` or __graft_entry__.build()")
        try:  # one HIP runtime per process: let torch's libamdhip64 load first
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return L


def check(rc, ctx=None):
    if rc != SK_OK:
        msg = ""
        if ctx:
            m = lib().sk_last_error(ctx)
            msg = m.decode() if m else ""
        raise StemKernelError(rc, msg)
    return rc


def default_params(kind=SU_STEM_STR, **over):
    p = KernelParams()
    lib().sk_kernel_params_default(C.byref(p), kind)
    for k, v in over.items():
        if k == "score_table":
            for i, t in enumerate(v):
                p.score_table[i] = float(t)
        else:
            setattr(p, k, v)
    return p
