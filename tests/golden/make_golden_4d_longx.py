"""Generate tests/golden/longx_4d.npz: 4-D stem kernel (full_dp) values for
long x against short y -- the column-group kernel holds x in LDS (sized per
launch from the batch's longest x, up to 2,048 residues), and x past that
limit goes to the span kernel (run_stem4d's col_ok).

Reference: StemKernel<double,BPMat>::full_dp stem_kernel/stem_kernel.cpp:282-351;
defaults of stem_kernel/main.cpp:46-64 (gap 0.8, stack 1.0, subst 0.5, loop 3,
bp_bound 0).  Expected values: the CPU oracle (oracle/sk_oracle.c; parity
against the reference's own output is unpinned).  The synthetic
fold's bytes are pinned by a SHA-256 stored beside the values.

Run:  python tests/golden/make_golden_4d_longx.py      (~1 min on 8 cores)
"""
import hashlib
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import stem_kernel_amd as ska  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def cases():
    """(x, y): |x| 640 / 700 / 1,200 (column kernel, x past the old fixed
    512-byte LDS region) against |y| 70 / 100 / 40, and |x| = 2,100 (past the
    column kernel's x limit: span kernel) against |y| = 24."""
    s = lambda L, k: ska.random_sequences(1, L, 0x5EED0500 + k)[0]
    return [(s(640, 1), s(70, 2)), (s(700, 3), s(100, 4)), (s(1200, 5), s(40, 6)),
            (s(2100, 7), s(24, 8))]


def _cell(c):
    a, b = c
    return po.stem4d(a.lower(), ska.fold(a.lower()), b.lower(), ska.fold(b.lower()),
                     float(np.float32(0.8)), 1.0, 0.5, 0.0, 0, 3, 0)


def main():
    cs = cases()
    with ProcessPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        vals = list(ex.map(_cell, cs))
    h = hashlib.sha256()
    for a, b in cs:
        for t in (a, b):
            h.update(np.ascontiguousarray(ska.fold(t.lower()), np.float64).tobytes())
    np.savez_compressed(os.path.join(HERE, "longx_4d.npz"), x=np.array([c[0] for c in cs]),
                        y=np.array([c[1] for c in cs]), value=np.array(vals), sha=np.array(h.hexdigest()))
    print(vals)


if __name__ == "__main__":
    main()
