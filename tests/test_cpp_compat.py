"""Drop-in check of include/stem_kernel_compat.hpp: a reference-shaped App
(tests/cpp/app_dropin.cpp -- App<K,LDF>::train / predict of
common/framework.h:100-306, written against KernelMatrix<double>,
SuStemStrKernel<double,MData>, DataLoaderFactory<DataLoader<MData> > and
BPMatrix::Options, with the include as the only change) compiles against the
compatibility header, and (GPU) produces the engine's Gram and predict rows
bit for bit."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "stem_kernel_amd")


def _build(tmp_path):
    exe = str(tmp_path / "app_dropin")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I",
                    os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "app_dropin.cpp"),
                    "-L", LIBDIR, "-lstem_kernel_amd", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_compat_app_compiles_and_links(tmp_path):
    assert os.path.exists(_build(tmp_path))


def _write_fa(path, seqs):
    with open(path, "w") as f:
        for k, s in enumerate(seqs):
            f.write(f">seq{k}\n{s[:40]}\n{s[40:]}\n")


@pytest.mark.gpu
@pytest.mark.parametrize("normalize", [0, 1])
def test_compat_app_matches_engine(gpu_ctx, tmp_path, normalize):
    import stem_kernel_amd as ska
    exe = _build(tmp_path)
    train = ska.random_sequences(6, 80, 0x5EED0001)
    # 12 test rows against one train set: the engine's dataset cache holds 8
    # sets, so the predict loop's single-row sets evict while the train set
    # is in use (a shared handle keeps it alive)
    test = ska.random_sequences(12, 75, 0x5EED0011)
    _write_fa(tmp_path / "train.fa", train)
    _write_fa(tmp_path / "test.fa", test)
    out = subprocess.run([exe, str(tmp_path / "train.fa"), str(tmp_path / "test.fa"),
                          str(tmp_path / "gram.libsvm"), str(normalize)], check=True,
                         capture_output=True, text=True, timeout=120).stdout.split("\n")
    n = len(train)
    gram = np.array([[float(v) for v in out[i].split()] for i in range(n)])
    rows = np.array([[float(v) for v in out[n + t].split()] for t in range(len(test))])
    kern = ska.SuStemStrKernel()
    # MData folds with the engine's GPU McCaskill (BPMatrix FOLD without ViennaRNA)
    ds = ska.Dataset.from_sequences(train, bpp=gpu_ctx.fold([s.lower() for s in train]))
    dt = ska.Dataset.from_sequences(test, bpp=gpu_ctx.fold([s.lower() for s in test]))
    assert np.array_equal(gram, gpu_ctx.gram(ds, kern, normalize=bool(normalize)))
    diag = gpu_ctx.diagonal(ds, kern)
    for t in range(len(test)):
        r, slf = gpu_ctx.test_row(dt, t, ds, kern, self_value=True)
        if normalize:
            r = r / np.sqrt(diag * slf)
        assert rows[t, 0] == slf
        assert np.array_equal(rows[t, 1:], r)
    lines = (tmp_path / "gram.libsvm").read_text().splitlines()
    assert len(lines) == n and lines[1].split()[:2] == ["-1", "0:2"]
