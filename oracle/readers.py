"""CPU restatement of the reference's example-file grammars (TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker of the product's
sk_seqfile_* readers, never by the product).

Each reader returns the examples DataLoader<MData>::get
(stem_kernel_lite/data.cpp:547-586) would pull from the text, as lists of rows.
The grammars are Boost.Spirit classic rules (parsed without a skipper):
kleene stars are greedy and never give characters back, alternatives are
tried in order, and a semantic action fires as soon as its sub-parser matches,
even when the enclosing rule then fails.  They are written here as regular
expressions whose character classes are disjoint where Spirit would not
backtrack (negative lookaheads where they are not).

Parity: the reference's readers need Boost.Spirit, absent from the image, so
this restatement is pinned by construction and by hand-derived expectations
in tests/test_readers.py ("parity unpinned" against the reference's output).
"""
from __future__ import annotations

import re
from typing import List

EOL = r"(?:\r\n|\r|\n)"
_eol = re.compile(EOL)


class FormatError(ValueError):
    pass


def _check_lengths(rows):
    # DataLoader<MData>::get (data.cpp:574-578)
    if any(len(r) != len(rows[0]) for r in rows):
        raise FormatError("wrong alignment")


# --------------------------------------------------------------- FASTA
# fa_parser (common/fa.cpp:13-55):
#   fa = head >> seq;  head = '>' >> *(blank_p | graph_p) >> eol_p
#   seq_l = *(graph_p - '>' - eol_p);  seq = +(seq_l[append_seq] >> eol_p)
_fa_head = re.compile(r">[ \t!-~]*" + EOL)
_fa_line = re.compile(r"[!-=?-~]*")  # graph_p without '>'


def read_fa(text: str) -> List[List[str]]:
    out, p = [], 0
    while True:
        m = _fa_head.match(text, p)
        if not m:
            break
        q, seq, lines = m.end(), "", 0
        while True:
            ln = _fa_line.match(text, q)
            seq += ln.group()  # append_seq fires before eol_p is tried
            e = _eol.match(text, ln.end())
            if not e:
                break
            q, lines = e.end(), lines + 1
        if not lines:
            break
        out.append([seq])
        p = q
    return out


# --------------------------------------------------------------- CLUSTAL
# aln_parser (common/aln.cpp:16-107):
#   aln = header >> +empty >> body;  head_word = "CLUSTAL" | "PROBCONS"
#   header = head_word >> +print_p >> eol_p;  empty = *blank_p >> eol_p
#   body_part = +seq[push_seq] >> !status
#   body = body_part[reset_index] >> *(+empty >> body_part[reset_index])
#   seq = (+graph_p - head_word)[name] >> +blank_p >> (+graph_p)[seq] >> *blank_p >> eol_p
#   status = *(chset("*:.") | blank_p) >> eol_p
_aln_header = re.compile(r"(?:CLUSTAL|PROBCONS)[ -~]+" + EOL)
_empty = re.compile(r"[ \t]*" + EOL)
_aln_seq = re.compile(r"([!-~]+)[ \t]+([!-~]+)[ \t]*" + EOL)
_aln_status = re.compile(r"[*:. \t]*" + EOL)


def _empties(text, p):
    n = 0
    while True:
        m = _empty.match(text, p)
        if not m:
            return p, n
        p, n = m.end(), n + 1


def _body_part(text, p, wa):
    k = 0
    while True:
        m = _aln_seq.match(text, p)
        if not m or m.group(1) in ("CLUSTAL", "PROBCONS"):  # +graph_p - head_word
            break
        name, seq = m.group(1), m.group(2)
        # push_seq (aln.cpp:40-54)
        if wa["i"] >= len(wa["names"]):
            wa["names"].append(name)
            wa["seqs"].append(seq)
        elif wa["names"][wa["i"]] == name:
            wa["seqs"][wa["i"]] += seq
        else:
            raise FormatError("format error: broken sequence name consistency")
        wa["i"] += 1
        p, k = m.end(), k + 1
    if not k:
        return None
    m = _aln_status.match(text, p)
    return m.end() if m else p


def _reset(wa):
    # reset_index (aln.cpp:56-72)
    if any(len(s) != len(wa["seqs"][0]) for s in wa["seqs"]):
        raise FormatError("format error: broken sequence length consistency")
    wa["i"] = 0


def read_aln(text: str) -> List[List[str]]:
    out, p = [], 0
    while True:
        m = _aln_header.match(text, p)
        if not m:
            break
        q, n = _empties(text, m.end())
        if not n:
            break
        wa = {"i": 0, "names": [], "seqs": []}
        q = _body_part(text, q, wa)
        if q is None:
            break
        _reset(wa)
        while True:
            r, n = _empties(text, q)
            if not n:
                break
            b = _body_part(text, r, wa)
            if b is None:
                break
            _reset(wa)
            q = b
        _check_lengths(wa["seqs"])
        out.append(wa["seqs"])
        p = q
    return out


# --------------------------------------------------------------- MAF
# maf_parser (common/maf.cpp:15-49):
#   maf = !header >> *(comment | empty) >> ali >> +seq >> *empty
#   header = "##maf" >> *print_p >> eol_p;  comment = comment_p("#")
#   ali = 'a' >> +blank_p >> *print_p >> eol_p
#   seq = ((seq_s1 >> seq_s2) | seq_i) >> eol_p
#   seq_s1 = 's' +blank +graph +blank uint +blank uint +blank
#   seq_s2 = sign +blank uint +blank (+graph)[push_back] *blank
#   seq_i = ('i' | 'e') +blank +print eol
_maf_header = re.compile(r"##maf[ -~]*" + EOL)
_maf_comment = re.compile(r"#[^\r\n]*(?:" + EOL + r"|\Z)")
_maf_ali = re.compile(r"a[ \t]+[ -~]*" + EOL)
_maf_s = re.compile(r"s[ \t]+[!-~]+[ \t]+(\d+)[ \t]+(\d+)[ \t]+[+-][ \t]+(\d+)[ \t]+([!-~]+)[ \t]*")
_maf_i = re.compile(r"[ie][ \t]+(?![ \t])[ -~]+" + EOL)


def _maf_block(text, p, rows):
    m = _maf_header.match(text, p)
    if m:
        p = m.end()
    while True:
        m = _maf_comment.match(text, p) or _empty.match(text, p)
        if not m or m.end() == p:
            break
        p = m.end()
    m = _maf_ali.match(text, p)
    if not m:
        return None
    p, k = m.end(), 0
    while True:
        m = _maf_s.match(text, p)
        if m and all(int(m.group(g)) <= 0xFFFFFFFF for g in (1, 2, 3)):
            rows.append(m.group(4))  # push_back_a fires before the eol
            e = _eol.match(text, m.end())
        else:
            m = _maf_i.match(text, p)
            e = _eol.match(text, m.end()) if m else None
        if not e:
            break
        p, k = e.end(), k + 1
    if not k:
        return None
    p, _ = _empties(text, p)
    return p


def read_maf(text: str) -> List[List[str]]:
    out, p = [], 0
    while True:
        rows = []
        q = _maf_block(text, p, rows)
        if q is None:
            break
        _check_lengths(rows)
        out.append(rows)
        p = q
    return out


def read(text: str, fmt: str) -> List[List[str]]:
    return {"fa": read_fa, "aln": read_aln, "maf": read_maf}[fmt](text)
