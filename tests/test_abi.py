"""The C ABI library loads and exports every symbol include/stem_kernel.h
declares; host-only entry points behave (no GPU needed)."""
import os
import re

import numpy as np
import pytest

import stem_kernel_amd as ska
from stem_kernel_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "stem_kernel.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sk_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported_and_bound():
    L = ska.lib()
    names = declared_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature"


def test_open_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        return
    try:
        ska.Context(0)
    except ska.StemKernelError as e:
        assert e.code in (-3, -2)
    else:
        raise AssertionError("sk_open succeeded without a GPU")


def test_params_defaults_match_reference_cli():
    # stem_kernel_lite/main.cpp:103-149
    p = ska.SuStemStrKernel().params
    assert (p.beta, p.loop_gap, p.alpha, p.gap, p.len_band) == (0.3, 0.2, 0.2, 0.8, 10)
    q = ska.SiStemStrKernel().params
    assert (q.stack, q.covar, q.match, q.mismatch) == (1.3, 0.8, 1.0, 0.8)


def test_libsvm_format_is_ostream_default():
    m = np.array([[1.0, 0.123456789, 1e-7], [123456789.0, 2.5, -0.0001]])
    txt = ska.format_libsvm(m, ["+1", "-1"])
    lines = txt.splitlines()
    assert lines[0] == "+1 0:1 1:1 2:0.123457 3:1e-07 "
    assert lines[1] == "-1 0:2 1:1.23457e+08 2:2.5 3:-0.0001 "


def test_random_sequences_deterministic():
    a = ska.random_sequences(3, 20, 0x5EED0002)
    b = ska.random_sequences(3, 20, 0x5EED0002)
    assert a == b and all(set(s) <= set("ACGU") and len(s) == 20 for s in a)


def test_dataset_errors():
    ds = ska.Dataset()
    try:
        ds.add("+1", ["ACGU", "ACG"], use_bp=False)  # rows of unequal length
    except ska.StemKernelError as e:
        assert e.code == -1
    else:
        raise AssertionError("wrong alignment accepted")
    assert len(ds) == 0


def test_kernel_matrix_save_compressed(tmp_path):
    """App's output (common/framework.h:138-160): .gz / .bz2 by file name."""
    import bz2
    import gzip
    km = ska.KernelMatrix.__new__(ska.KernelMatrix)  # no GPU context needed to write
    km.matrix = np.array([[1.0, 0.5], [0.5, 1.0]])
    km.label = ["+1", "-1"]
    want = ska.format_libsvm(km.matrix, km.label)
    km.save(str(tmp_path / "k.txt"))
    km.save(str(tmp_path / "k.txt.gz"))
    km.save(str(tmp_path / "k.txt.bz2"))
    assert (tmp_path / "k.txt").read_text() == want
    assert gzip.open(tmp_path / "k.txt.gz", "rt").read() == want
    assert bz2.open(tmp_path / "k.txt.bz2", "rt").read() == want
    with pytest.raises(ska.StemKernelError, match="cannot open"):
        km.save(str(tmp_path / "missing" / "k.txt"))
