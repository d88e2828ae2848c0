"""Drop-in checks of the per-tool compatibility headers: reference-shaped
mains of the other three tools -- the 4-D stem kernel (stem_kernel/main.cpp:
88-160, include/stem_kernel_ref_compat.hpp), the naive string kernel
(string_kernel/main.cpp:73-112, include/string_kernel_compat.hpp) and the
BPLA kernel (bpla_kernel/main.cpp:100-127, include/bpla_kernel_compat.hpp) --
compile against the headers with the include as the only engine-specific
line (CPU) and produce the engine's values bit for bit (GPU).  The legacy
Fasta reader's quirks (common/fasta.cpp) are checked on CPU."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "stem_kernel_amd")
MAINS = ["ref4d_dropin", "naive_dropin", "bpla_dropin", "fasta_quirks"]


def _build(tmp_path, name):
    exe = str(tmp_path / name)
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", name + ".cpp"), "-L", LIBDIR, "-lstem_kernel_amd",
                    f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("name", MAINS)
def test_dropin_main_compiles(tmp_path, name):
    assert os.path.exists(_build(tmp_path, name))


def test_headers_are_self_contained(tmp_path):
    for h in ("stem_kernel_compat.hpp", "stem_kernel_ref_compat.hpp", "string_kernel_compat.hpp",
              "bpla_kernel_compat.hpp"):
        src = tmp_path / "inc.cpp"
        src.write_text(f'#include "{h}"\nint main() {{ return 0; }}\n')
        subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-I",
                        os.path.join(ROOT, "include"), str(src)], check=True)


def test_fasta_reader_quirks(tmp_path):
    """common/fasta.cpp: text before the first '>' is skipped; the name is
    the first line, the sequence the whitespace-joined rest, one trailing
    '*' dropped; a file ending in a bare '>' repeats the last sequence
    (GetNextSeq returns "" -- non-null -- and leaves m_seq in place); the
    example loader lowercases (common/example.cpp:27-35)."""
    exe = _build(tmp_path, "fasta_quirks")
    fa = tmp_path / "q.fa"
    fa.write_text("junk line\n>a  desc\nAC GU\nUU*\n>b\nGG\n\n>  c\nAUG\n>")
    lines = tmp_path / "q.txt"
    lines.write_text("+1 ACGU\n-1\n-1 GGaa extra\n")
    out = subprocess.run([exe, str(fa), str(lines)], check=True, capture_output=True, text=True).stdout
    assert out.splitlines() == ["+1\tacguuu", "+1\tgg", "+1\taug", "+1\taug", "+1\tacgu", "-1\tggaa"]
    fa.write_text(">x\nACGU")  # no trailing newline, no trailing '>'
    out = subprocess.run([exe, str(fa)], check=True, capture_output=True, text=True).stdout
    assert out.splitlines() == ["+1\tacgu"]


def _fa(path, seqs):
    with open(path, "w") as f:
        for k, s in enumerate(seqs):
            f.write(f">s{k}\n{s}\n")


def _matrix(lines, rows):
    return np.array([[float(v) for v in lines[i].split()] for i in range(rows)])


@pytest.mark.gpu
@pytest.mark.parametrize("use_gu,band,normalize", [(0, 0, 0), (1, 0, 1), (0, 5, 0)])
def test_ref4d_dropin_matches_engine(gpu_ctx, tmp_path, use_gu, band, normalize):
    import stem_kernel_amd as ska
    exe = _build(tmp_path, "ref4d_dropin")
    train = ska.random_sequences(5, 36, 0x5EED0021)
    test = ska.random_sequences(3, 30, 0x5EED0022)
    _fa(tmp_path / "tr.fa", train)
    _fa(tmp_path / "te.fa", test)
    low = [s.lower() for s in train]
    tlow = [s.lower() for s in test]
    # BPMatrix model: every sequence folded with noGU = use_GU (PFWrapper(seq, useGU))
    ds = ska.Dataset.from_sequences(low, bpp=gpu_ctx.fold(low, no_gu=bool(use_gu)), th=1.0)
    dt = ska.Dataset.from_sequences(tlow, bpp=gpu_ctx.fold(tlow, no_gu=bool(use_gu)), th=1.0)
    kern = ska.StemKernel4D(bp_bound=0.0, band=band)
    out = subprocess.run([exe, str(tmp_path / "g.txt"), "", "0.0", str(use_gu), str(band), "0.0", str(normalize),
                          str(tmp_path / "tr.fa")], check=True, capture_output=True, text=True,
                         timeout=300).stdout.splitlines()
    got = _matrix(out, len(train))
    assert np.array_equal(got, gpu_ctx.gram(ds, kern, normalize=bool(normalize)))
    raw = gpu_ctx.gram(ds, kern)
    assert float(out[len(train)].split()[1]) == raw[0, 1]  # Kernel::operator() on one pair
    # test x train with norms
    out = subprocess.run([exe, str(tmp_path / "g.txt"), "norms", "0.0", str(use_gu), str(band), "0.0",
                          str(normalize), str(tmp_path / "tr.fa"), str(tmp_path / "te.fa")], check=True,
                         capture_output=True, text=True, timeout=300).stdout.splitlines()
    m, s = gpu_ctx.test_matrix(dt, ds, kern, norm_test=True, normalize=bool(normalize))
    assert np.array_equal(_matrix(out, len(test)), m)
    assert np.array_equal(np.array([float(v) for v in out[len(test):2 * len(test)]]), s)


@pytest.mark.gpu
@pytest.mark.parametrize("use_gu", [0, 1])
def test_ref4d_dropin_basepair_models_give_one(gpu_ctx, tmp_path, use_gu):
    """Normal / Wobble models with the CLI's bp_bound 1.0: K = 1 for every
    pair."""
    import stem_kernel_amd as ska
    exe = _build(tmp_path, "ref4d_dropin")
    _fa(tmp_path / "tr.fa", ska.random_sequences(4, 30, 0x5EED0023))
    out = subprocess.run([exe, str(tmp_path / "g.txt"), "", "1.0", str(use_gu), "0", "0.0", "0",
                          str(tmp_path / "tr.fa")], check=True, capture_output=True, text=True,
                         timeout=300).stdout.splitlines()
    assert np.all(_matrix(out, 4) == 1.0)


@pytest.mark.gpu
@pytest.mark.parametrize("normalize", [0, 1])
def test_naive_dropin_matches_engine(gpu_ctx, tmp_path, normalize):
    import stem_kernel_amd as ska
    exe = _build(tmp_path, "naive_dropin")
    train = ska.random_sequences(6, 80, 0x5EED0024)
    _fa(tmp_path / "tr.fa", train)
    out = subprocess.run([exe, str(tmp_path / "g.txt"), "0.75", str(normalize), str(tmp_path / "tr.fa")],
                         check=True, capture_output=True, text=True, timeout=300).stdout.splitlines()
    ds = ska.Dataset.from_sequences([s.lower() for s in train])
    kern = ska.NaiveStringKernel(gap=0.75)
    assert np.array_equal(_matrix(out, 6), gpu_ctx.gram(ds, kern, normalize=bool(normalize)))
    assert float(out[6].split()[1]) == gpu_ctx.gram(ds, kern)[0, 1]


@pytest.mark.gpu
@pytest.mark.parametrize("nobp,sw", [(0, 0), (1, 0), (0, 1)])
def test_bpla_dropin_matches_engine(gpu_ctx, tmp_path, nobp, sw):
    import stem_kernel_amd as ska
    exe = _build(tmp_path, "bpla_dropin")
    train = ska.random_sequences(5, 60, 0x5EED0025)
    _fa(tmp_path / "tr.fa", train)
    out = subprocess.run([exe, str(tmp_path / "g.txt"), str(nobp), str(sw), "0", str(tmp_path / "tr.fa")],
                         check=True, capture_output=True, text=True, timeout=300).stdout.splitlines()
    low = [s.lower() for s in train]
    ds = ska.Dataset.from_sequences(train, bpp=None if nobp else gpu_ctx.fold(low), th=1.0)
    kern = ska.BPLAKernel(noBP=bool(nobp), SW=bool(sw))
    g = gpu_ctx.gram(ds, kern)
    assert np.array_equal(_matrix(out, 5), g)
    assert float(out[5].split()[1]) == g[0, 1]
    if not nobp and not sw:
        v, d = gpu_ctx.bpla_gradients(ds, ska.BPLAKernel(), np.array([0]), np.array([1]))
        got = [float(t) for t in out[6].split()[1:]]
        assert got[0] == v[0] and got[1:] == list(d[0])
