"""Example-file readers (FASTA / CLUSTAL / MAF, the formats
DataLoader<MData>::get pulls examples from, stem_kernel_lite/data.cpp:547-586).

The product's C++ scanners (sk_seqfile_*, csrc/host/readers.cpp) against the
regex restatement in oracle/readers.py and against expectations derived by
hand from the reference grammars (common/fa.cpp:13-55, aln.cpp:16-107,
maf.cpp:15-49).  The reference readers need Boost.Spirit, absent here:
parity unpinned against the reference's own output, pinned by construction.
The parsing tests are host code (no GPU); one GPU test runs a file end to end."""
import numpy as np
import pytest

import stem_kernel_amd as ska
from oracle import readers as orr


def both(text, fmt):
    got = ska.parse_examples(text, fmt)
    assert got == orr.read(text, fmt)
    return got


# ---------------------------------------------------------------- FASTA
def test_fasta_records_and_line_joining():
    t = ">s1 a description\nACGU\nGG-U\n\n>s2\r\nAAA\r\nCC\r>s3\nU\n"
    assert both(t, "fa") == [["ACGUGG-U"], ["AAACC"], ["U"]]


def test_fasta_quirks():
    # a blank inside a sequence line ends the record's lines there; the part
    # before the blank was already appended, the rest stops the reader
    assert both(">a\nAC\nGG UU\n>b\nA\n", "fa") == [["ACGG"]]
    # the final line needs its newline ...
    assert both(">a\nACGU", "fa") == []
    # ... unless an earlier line had one: the unterminated tail is appended
    assert both(">a\nAC\nGU", "fa") == [["ACGU"]]
    # a header without a newline, or leading junk, reads nothing
    assert both(">a", "fa") == [] and both("x\n>a\nA\n", "fa") == []
    assert both("", "fa") == []


# ---------------------------------------------------------------- CLUSTAL
ALN = """CLUSTAL W (1.83) multiple sequence alignment

s1      ACGU-A
s2      ACG-UA
        *** *

s1      GGC
s2      GGA
        **
"""


def test_clustal_blocks():
    assert both(ALN, "aln") == [["ACGU-AGGC", "ACG-UAGGA"]]
    # PROBCONS header, several alignments back to back
    two = ALN + ALN.replace("CLUSTAL W (1.83)", "PROBCONS version 1.1").replace("ACG", "UUU")
    assert both(two, "aln") == [["ACGU-AGGC", "ACG-UAGGA"], ["UUUU-AGGC", "UUU-UAGGA"]]


def test_clustal_quirks():
    # no conservation line: !status eats the single blank separator, so the
    # second block needs two blank lines to be read
    one = "CLUSTAL x\n\na AC\nb AG\n\na GG\nb GU\n"
    assert both(one, "aln") == [["AC", "AG"]]
    assert both(one.replace("AG\n\n", "AG\n\n\n"), "aln") == [["ACGG", "AGGU"]]
    # "CLUSTAL" alone on the header line: +print_p needs a character
    assert both("CLUSTAL\n\na AC\n", "aln") == []
    # a sequence named exactly like a head word ends the block
    assert both("CLUSTAL x\n\na AC\nCLUSTAL AG\n", "aln") == [["AC"]]
    assert both("CLUSTAL x\n\na AC\nCLUSTALW AG\n", "aln") == [["AC", "AG"]]
    # trailing column counts end the block at that line
    assert both("CLUSTAL x\n\na AC 2\nb AG 2\n", "aln") == []


def test_clustal_format_errors():
    with pytest.raises(ska.StemKernelError, match="name consistency"):
        ska.parse_examples("CLUSTAL x\n\na AC\nb AG\n\n\nb GG\na GU\n", "aln")
    with pytest.raises(orr.FormatError):
        orr.read_aln("CLUSTAL x\n\na AC\nb AG\n\n\nb GG\na GU\n")
    with pytest.raises(ska.StemKernelError, match="length consistency"):
        ska.parse_examples("CLUSTAL x\n\na ACG\nb AG\n", "aln")


# ---------------------------------------------------------------- MAF
MAF = """##maf version=1 scoring=none
# a comment

a score=10.0
s hg18.chr1 100 6 + 1000 ACGU-A
s mm9.chr2  200 6 - 2000 ACG-UA

a score=3
s x 0 3 + 3 AAA
s y 0 3 + 3 CCC
"""


def test_maf_blocks():
    assert both(MAF, "maf") == [["ACGU-A", "ACG-UA"], ["AAA", "CCC"]]


def test_maf_quirks():
    # an i/e line must be followed by an empty line (seq_i has its own eol_p)
    t = "a x\ns a 0 2 + 2 AC\ni a N 0 C 0\n\ns b 0 2 + 2 AG\n"
    assert both(t, "maf") == [["AC", "AG"]]
    t = "a x\ns a 0 2 + 2 AC\ni a N 0 C 0\ns b 0 2 + 2 AG\n"
    assert both(t, "maf") == [["AC"]]
    # 'a' needs a blank after it
    assert both("a\ns a 0 2 + 2 AC\n", "maf") == []
    # the row is pushed before its eol is seen: a junk tail still yields it
    assert both("a x\ns a 0 2 + 2 AC\ns b 0 2 + 2 AG junk\n", "maf") == [["AC", "AG"]]
    # counts past 2^32-1 fail uint_p
    assert both("a x\ns a 0 99999999999 + 2 AC\n", "maf") == []


def test_wrong_alignment():
    with pytest.raises(ska.StemKernelError, match="wrong alignment"):
        ska.parse_examples("a x\ns a 0 2 + 2 AC\ns b 0 2 + 2 AGU\n", "maf")


# ---------------------------------------------------------------- fuzz
_FRAGS = {
    "fa": [">n d\n", ">x\r\n", "ACGU\n", "GG-U\n", "\n", "AC GU\n", "UU", ">", "A\r", "N\n"],
    "aln": ["CLUSTAL W x\n", "PROBCONS v\n", "\n", "  \n", "a AC\n", "b AG\n", "a GU\n",
            "b UU\n", "   **\n", "CLUSTAL AC\n", "c A\n", "a AC 4\n", "\t\n"],
    "maf": ["##maf v=1\n", "# c\n", "\n", "a s=1\n", "a\n", "s a 0 2 + 9 AC\n",
            "s b 1 2 - 9 AG\n", "i a N 0 C 0\n", "e a 0 2 + 9 I\n", "s c 0 2 + 9 AC x\n", "q\n"],
}


@pytest.mark.parametrize("fmt", ["fa", "aln", "maf"])
def test_fuzz_against_restatement(fmt):
    rng = np.random.default_rng({"fa": 1, "aln": 2, "maf": 3}[fmt])
    frags = _FRAGS[fmt]
    for _ in range(1500):
        text = "".join(frags[i] for i in rng.integers(len(frags), size=rng.integers(1, 14)))
        try:
            want = orr.read(text, fmt)
        except orr.FormatError:
            with pytest.raises(ska.StemKernelError):
                ska.parse_examples(text, fmt)
            continue
        assert ska.parse_examples(text, fmt) == want, repr(text)


def test_read_file_and_dataset(tmp_path):
    p = tmp_path / "x.fa"
    p.write_text(">a\nACGUACGGAAACCGU\n>b\nGGGAAAUCCCGGUAA\n")
    assert ska.read_examples(str(p), "fa") == [["ACGUACGGAAACCGU"], ["GGGAAAUCCCGGUAA"]]
    ds = ska.Dataset()
    assert ds.add_file("+1", str(p), "fa") == 2 and len(ds) == 2
    with pytest.raises(ska.StemKernelError, match="no such file"):
        ska.read_examples(str(tmp_path / "missing.fa"))


@pytest.mark.gpu
def test_clustal_file_to_gram(gpu_ctx, tmp_path):
    """End to end: a CLUSTAL file through the reader, the synthetic fold and
    the GPU Gram, against the oracle on the same rows (1e-6 relative)."""
    from oracle import pyoracle as po
    from tests.helpers import make_examples, mutate_alignment, rel_err
    alns = [mutate_alignment(s, 3, 40 + k) for k, s in enumerate(ska.random_sequences(4, 60, 77))]
    text = ""
    for a in alns:
        text += "CLUSTAL W (1.83) multiple sequence alignment\n\n"
        for off in range(0, 60, 25):
            text += "".join(f"r{r}   {row[off:off + 25]}\n" for r, row in enumerate(a)) + "     *\n"
            text += "\n" if off + 25 < 60 else ""
    p = tmp_path / "x.aln"
    p.write_text(text)
    got_rows = ska.read_examples(str(p), "aln")
    assert got_rows == [list(a) for a in alns]
    ds = ska.Dataset()
    ds.add_file("+1", str(p), "aln")
    _, om = make_examples(got_rows)
    kern = ska.SuStemStrKernel()
    K = gpu_ctx.gram(ds, kern)
    n = len(alns)
    ref = np.array([[po.kernel_value(kern.params.kind, om[min(i, j)], om[max(i, j)], kern.params)
                     for j in range(n)] for i in range(n)])
    assert rel_err(K, ref) < 1e-6
