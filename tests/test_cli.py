"""The stem_kernel_lite CLI (stem_kernel_amd/bin/stem_kernel_lite, built from
csrc/cli/stem_kernel_lite.cpp over include/stem_kernel_compat.hpp): the
reference's flag surface (stem_kernel_lite/main.cpp:85-151, common/framework.cpp:12-46),
positional layout (Options::parse_extra_args, framework.cpp:48-93), console
messages and libsvm outputs (KernelMatrix::print, Output::kernel_output /
norm_output).

CPU tests: usage, refused options, error messages.  GPU tests: train and
predict outputs against the engine through Python on the same GPU-folded
examples (libsvm text holds 6 significant digits: 1e-5 relative)."""
import gzip
import os
import subprocess

import numpy as np
import pytest

import stem_kernel_amd as ska

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "stem_kernel_amd", "bin", "stem_kernel_lite")


def _run(args, **kw):
    return subprocess.run([CLI] + [str(a) for a in args], capture_output=True, text=True,
                          timeout=300, **kw)


def _write_fa(path, seqs):
    with open(path, "w") as f:
        for k, s in enumerate(seqs):
            f.write(f">s{k}\n{s}\n")


def _parse_libsvm(text):
    labels, rows = [], []
    for line in text.splitlines():
        tok = line.split()
        labels.append(tok[0])
        rows.append([float(t.split(":")[1]) for t in tok[2:]])
    return labels, np.array(rows)


def test_cli_built():
    assert os.access(CLI, os.X_OK)


def test_usage_without_arguments():
    r = _run([])
    assert r.returncode == 1
    assert "Kernel Matrix Calculator for Stem Kernels" in r.stdout
    for flag in ("--basepair", "--loop-gap", "--length-band", "--no-string", "--noGU", "--normalize"):
        assert flag in r.stdout


@pytest.mark.parametrize("flag,msg", [("--use-alifold", "use-alifold")])
def test_refused_folding_options(tmp_path, flag, msg):
    _write_fa(tmp_path / "a.fa", ["GGGGAAACCCC"])
    r = _run([tmp_path / "o.txt", "+1", tmp_path / "a.fa", flag])
    assert r.returncode == 1 and msg in r.stdout


def test_predict_needs_model(tmp_path):
    _write_fa(tmp_path / "a.fa", ["GGGGAAACCCC"])
    r = _run([tmp_path / "o.txt", "+1", tmp_path / "a.fa", "--test", "+1", tmp_path / "a.fa",
              "--predict", tmp_path / "p"])
    assert r.returncode == 1 and "--model" in r.stdout


def test_missing_file_message(tmp_path):
    r = _run([tmp_path / "o.txt", "+1", tmp_path / "missing.fa"])
    assert r.returncode == 1 and "missing.fa: no such file" in r.stdout


def test_bad_option_value(tmp_path):
    r = _run(["-p", "abc", tmp_path / "o.txt", "+1", tmp_path / "a.fa"])
    assert r.returncode == 1 and "invalid" in r.stderr


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def fa_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("cli")
    pos = ska.random_sequences(4, 70, 0x5EED0501)
    neg = ska.random_sequences(3, 65, 0x5EED0502)
    test = ska.random_sequences(2, 60, 0x5EED0503)
    _write_fa(d / "pos.fa", pos)
    _write_fa(d / "neg.fa", neg)
    _write_fa(d / "test.fa", test)
    return d, pos, neg, test


KERNELS = {(): ska.SuStemStrKernel(), ("--no-string",): ska.SuStemKernel(),
           ("--no-ribosum",): ska.SiStemStrKernel(), ("--no-string", "--no-ribosum"): ska.SiStemKernel(),
           ("--log",): ska.LSuStemStrKernel(), ("--log", "--no-string"): ska.LSuStemKernel()}


@pytest.mark.gpu
@pytest.mark.parametrize("flags", sorted(KERNELS))
def test_cli_train_matches_engine(gpu_ctx, fa_files, flags):
    d, pos, neg, _ = fa_files
    out = d / ("train_" + "_".join(f.strip("-") for f in flags) + ".txt")
    r = _run(list(flags) + ["-n", out, "+1", d / "pos.fa", "-1", d / "neg.fa"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"loading {d / 'pos.fa'} as label +1" in r.stdout and "elapsed time:" in r.stdout
    labels, got = _parse_libsvm(out.read_text())
    assert labels == ["+1"] * 4 + ["-1"] * 3
    ds = ska.Dataset.folded(gpu_ctx, pos + neg, labels=labels)
    ref = gpu_ctx.gram(ds, KERNELS[flags], normalize=True)
    # log kernels can be negative: normalising takes sqrt of a negative
    # diagonal (NaN), in the reference and here alike
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.max(np.abs(got[ok] - ref[ok]) / np.maximum(np.abs(ref[ok]), 1e-300)) < 1e-5


@pytest.mark.gpu
def test_cli_train_gz_and_options(gpu_ctx, fa_files):
    d, pos, neg, _ = fa_files
    out = d / "gram.txt.gz"
    r = _run(["--basepair", "0.02", "-b", "0.4", "--loop-gap=0.3", "-G", "0.7", "--length-band", "8",
              "--noGU", out, "+1", d / "pos.fa"])
    assert r.returncode == 0, r.stdout + r.stderr
    labels, got = _parse_libsvm(gzip.open(out, "rt").read())
    ds = ska.Dataset.folded(gpu_ctx, pos, th=0.02, no_gu=True)
    ref = gpu_ctx.gram(ds, ska.SuStemStrKernel(beta=0.4, loop_gap=0.3, gap=0.7, len_band=8))
    assert np.max(np.abs(got - ref) / np.abs(ref)) < 1e-5


@pytest.mark.gpu
def test_cli_no_lonely_pairs(gpu_ctx, fa_files):
    """--noLonelyPairs (common/bpmatrix.cpp:56-58, 149) reaches the fold: the
    Gram is the one of examples folded with SK_FOLD_NO_LONELY_PAIRS."""
    d, pos, neg, _ = fa_files
    out = d / "gram_nolp.txt"
    r = _run(["--noLonelyPairs", out, "+1", d / "pos.fa"])
    assert r.returncode == 0, r.stdout + r.stderr
    _, got = _parse_libsvm(out.read_text())
    ds = ska.Dataset.folded(gpu_ctx, pos, no_lonely_pairs=True)
    ref = gpu_ctx.gram(ds, ska.SuStemStrKernel())
    assert np.max(np.abs(got - ref) / np.abs(ref)) < 1e-5


@pytest.mark.gpu
def test_cli_train_bz2_equals_plain(gpu_ctx, fa_files):
    """`.bz2` output (common/framework.h:142-147's bzip2 filter) holds the
    same text as the plain file."""
    import bz2
    d, pos, neg, _ = fa_files
    plain, packed = d / "gram_plain.txt", d / "gram_packed.txt.bz2"
    for out in (plain, packed):
        r = _run(["-n", out, "+1", d / "pos.fa", "-1", d / "neg.fa"])
        assert r.returncode == 0, r.stdout + r.stderr
    assert bz2.open(packed, "rt").read() == plain.read_text()


@pytest.mark.gpu
def test_cli_predict_rows_and_norms(gpu_ctx, fa_files, tmp_path):
    d, pos, neg, test = fa_files
    out, norms = tmp_path / "rows.txt", tmp_path / "norms.txt"
    # a libsvm model whose SV section names training examples 2 and 5 (1-based)
    model = tmp_path / "model"
    model.write_text("svm_type c_svc\nkernel_type precomputed\nnr_class 2\ntotal_sv 2\n"
                     "rho 0.1\nlabel 1 -1\nnr_sv 1 1\nSV\n0.5 0:2 \n-0.5 0:5 \n")
    r = _run(["-n", "-x", norms, "--model", model, out, "+1", d / "pos.fa", "-1", d / "neg.fa",
              "--test", "+1", d / "test.fa"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"predicting {d / 'test.fa'}" in r.stdout and "elapsed time for diagonals" in r.stdout
    labels, got = _parse_libsvm(out.read_text())
    assert labels == ["+1", "+1"]
    lines = out.read_text().splitlines()
    assert lines[0].split()[1] == "0:1" and lines[1].split()[1] == "0:2"
    train = ska.Dataset.folded(gpu_ctx, pos + neg)
    tst = ska.Dataset.folded(gpu_ctx, test)
    kern = ska.SuStemStrKernel()
    sv = np.array([1, 4], np.int32)
    diag = gpu_ctx.diagonal(train, kern, sv_index=sv)
    self_vals = []
    for t in range(len(test)):
        row, slf = gpu_ctx.test_row(tst, t, train, kern, sv_index=sv, self_value=True)
        with np.errstate(invalid="ignore", divide="ignore"):  # non-SV entries: 0 / 0, as in the reference
            ref = row / np.sqrt(diag * slf)
        self_vals.append(slf)
        nz = np.isin(np.arange(len(row)), sv)
        assert np.max(np.abs(got[t][nz] - ref[nz]) / np.abs(ref[nz])) < 1e-5
    nrm = np.array([float(v) for v in norms.read_text().split()])
    assert np.max(np.abs(nrm - np.array(self_vals)) / np.array(self_vals)) < 1e-5


@pytest.mark.gpu
def test_cli_predict_with_svm_models(gpu_ctx, fa_files, tmp_path):
    """--model/--predict pairs: Output::prob_output through SVMPredict
    (framework.cpp:211-221, libsvm/svm_util.cpp:11-80) on the normalised
    test rows; a C-SVC model with probabilities and an epsilon-SVR model,
    both trained by scikit-learn's libsvm on the engine's Gram."""
    svm = pytest.importorskip("sklearn.svm")
    from oracle import svm_oracle as so
    d, pos, neg, test = fa_files
    train = ska.Dataset.folded(gpu_ctx, pos + neg)
    tst = ska.Dataset.folded(gpu_ctx, test)
    kern = ska.SuStemStrKernel()
    K = gpu_ctx.gram(train, kern, normalize=True)
    y = np.array([1] * len(pos) + [-1] * len(neg))
    clf = svm.SVC(kernel="precomputed", C=4.0, probability=True, random_state=0).fit(K, y)
    reg = svm.SVR(kernel="precomputed", C=2.0, epsilon=0.01).fit(K, np.linspace(0, 1, len(y)))
    mc = dict(svm_type="c_svc", nr_class=2, label=[int(c) for c in clf.classes_],
              nSV=clf.n_support_.tolist(), sv_index=(clf.support_ + 1).tolist(),
              sv_coef=np.atleast_2d(clf._dual_coef_).tolist(), rho=(-clf._intercept_).tolist(),
              probA=clf.probA_.tolist(), probB=clf.probB_.tolist())
    mr = dict(svm_type="epsilon_svr", nr_class=2, sv_index=(reg.support_ + 1).tolist(),
              sv_coef=np.atleast_2d(reg._dual_coef_).tolist(), rho=(-reg._intercept_).tolist())
    so.write_model(tmp_path / "mc", mc)
    so.write_model(tmp_path / "mr", mr)
    r = _run(["-n", "--no-matrix", "--model", tmp_path / "mc", "--predict", tmp_path / "pc",
              "--model", tmp_path / "mr", "--predict", tmp_path / "pr", tmp_path / "rows.txt",
              "+1", d / "pos.fa", "-1", d / "neg.fa", "--test", "-1", d / "test.fa"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert not (tmp_path / "rows.txt").exists()  # --no-matrix
    pc = (tmp_path / "pc").read_text().splitlines()
    pr = (tmp_path / "pr").read_text().splitlines()
    assert pc[0].split() == ["labels"] + [str(c) for c in clf.classes_]
    assert pr[0].split() == ["labels", "0", "0"]  # an SVR model has no labels
    sv = np.union1d(clf.support_, reg.support_).astype(np.int32)
    diag = gpu_ctx.diagonal(train, kern, sv_index=sv)
    for t in range(len(test)):
        row, slf = gpu_ctx.test_row(tst, t, train, kern, sv_index=sv, self_value=True)
        with np.errstate(invalid="ignore", divide="ignore"):
            row = row / np.sqrt(diag * slf)
        lab, prob = so.predict_probability(mc, row)
        got = [float(v) for v in pc[t + 1].split()]
        assert got[0] == lab and np.allclose(got[1:], prob, rtol=1e-5, atol=1e-6)
        dec = so.decision_values(mr, row)
        got = [float(v) for v in pr[t + 1].split()]
        assert got[0] == -1.0 and np.allclose(got[1:], dec, rtol=1e-5, atol=1e-6)
