"""The C++ facade (include/stem_kernel.hpp) as a reference-side caller would
use it: compile a KernelMatrix::calculate + print program against the C ABI,
then (GPU) check its libsvm output against the oracle."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "stem_kernel_amd")


def _build(tmp_path):
    exe = str(tmp_path / "gram_facade")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "gram_facade.cpp"), "-L", LIBDIR,
                    "-lstem_kernel_amd", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_facade_compiles_and_links(tmp_path):
    assert os.path.exists(_build(tmp_path))


def _parse_libsvm(text, n):
    m = np.zeros((n, n))
    labels = []
    for i, line in enumerate(text.strip().splitlines()):
        tok = line.split()
        labels.append(tok[0])
        assert tok[1] == f"0:{i + 1}"
        for t in tok[2:]:
            j, v = t.split(":")
            m[i, int(j) - 1] = float(v)
    return labels, m


@pytest.mark.gpu
def test_facade_gram_matches_oracle(tmp_path):
    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    n, L, seed = 5, 60, 0x5EED0001
    exe = _build(tmp_path)
    out = subprocess.run([exe, str(n), str(L), hex(seed)], check=True, capture_output=True,
                         text=True, timeout=120).stdout
    labels, m = _parse_libsvm(out, n)
    assert labels == ["+1", "-1", "+1", "-1", "+1"]
    seqs = ska.random_sequences(n, L, seed)
    om = [po.OMData([s], [ska.fold(s)], 0.01) for s in seqs]
    p = ska.SuStemStrKernel().params
    ref = np.zeros((n, n))
    for i in range(n):
        for j in range(i, n):
            ref[i, j] = ref[j, i] = po.kernel_value(p.kind, om[i], om[j], p)
    # text carries 6 significant digits (ostream default)
    np.testing.assert_allclose(m, ref, rtol=6e-6)
