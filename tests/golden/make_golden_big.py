"""Generate tests/golden/big_dag.npz: oracle values for y examples beyond the
DAG stem kernel's register classes (sk_dag_stem_big_kernel, dag_stem_big.hip).

* Two sequences of L = 500 (synthetic fold: 2,158-2,223 non-leaf nodes, over
  the 2,048 the register classes hold) and one of L = 300 (a register-class
  example), all ordered pairs, so calls mix both kernels.
* A caller-supplied bpp with a stem edge of 1,077 skipped positions (gaps
  beyond the packed 10-bit field): L = 1,100, pairs (1, 1100) and
  (501, 521) (1-based, p = 0.5 each) plus a short helix.

Reference: StemKernel<ST,MData>::operator() stem_kernel_lite/stem_kernel.cpp:14-95
(no size limit).  Expected values come from the CPU oracle
(oracle/sk_oracle.c, a line-by-line restatement; parity against the
reference's own output is unpinned); the synthetic fold's
bytes are pinned by a SHA-256 stored beside the values.

Run:  python tests/golden/make_golden_big.py      (~1 min on 8 cores)
"""
import hashlib
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import stem_kernel_amd as ska  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

KINDS = (0, 1, 2, 3)  # SuStem, SiStem, SuStr, SiStr


def big_seqs():
    return ska.random_sequences(2, 500, 0x5EED0106) + ska.random_sequences(1, 300, 0x5EED0107)


def gap_case():
    """(sequence, packed upper-triangular bpp) with a 1,077-gap stem edge."""
    L = 1100
    seq = ska.random_sequences(1, L, 0x5EED0108)[0]
    bpp = np.zeros(L * (L - 1) // 2)

    def put(i, j, p):  # 0-based i < j, row-major upper triangle without diagonal
        bpp[i * L - i * (i + 1) // 2 + (j - i - 1)] = p
    put(0, L - 1, 0.5)
    put(500, 520, 0.5)
    for k in range(4):  # a short helix inside the hairpin side
        put(502 + k, 518 - k, 0.3)
    return seq, bpp


_OM = {}


def _cell(args):
    kind, i, j = args
    if not _OM:
        for k, s in enumerate(big_seqs()):
            _OM[k] = po.OMData([s], [ska.fold(s.lower())], 0.01)
        seq, bpp = gap_case()
        _OM["gap"] = po.OMData([seq], [bpp], 0.01)
    p = ska.SuStemStrKernel().params
    return po.kernel_value(kind, _OM[i], _OM[j], p)


def main():
    seqs = big_seqs()
    n = len(seqs)
    arrays = {"seqs": np.array(seqs)}
    h = hashlib.sha256()
    for s in seqs:
        h.update(np.ascontiguousarray(ska.fold(s.lower()), np.float64).tobytes())
    arrays["sha"] = np.array(h.hexdigest())
    with ProcessPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        for kind in KINDS:
            cells = [(kind, i, j) for i in range(n) for j in range(n)]
            arrays[f"K{kind}"] = np.array(list(ex.map(_cell, cells, chunksize=1))).reshape(n, n)
            print("kind", kind, flush=True)
        gseq, gbpp = gap_case()
        arrays["gap_seq"] = np.array(gseq)
        arrays["gap_bpp"] = gbpp
        for kind in (0, 1):
            arrays[f"gap_K{kind}"] = np.array(
                list(ex.map(_cell, [(kind, "gap", "gap"), (kind, 0, "gap"), (kind, "gap", 2)])))
    np.savez_compressed(os.path.join(HERE, "big_dag.npz"), **arrays)


if __name__ == "__main__":
    main()
