"""Generate tests/golden/long_4d.npz: 4-D stem kernel values for sequences
the register layout of one 512-cell k tile cannot hold (|y| >= 512: the
kernel sweeps k tiles right to left, stem4d.hip), plus a long x.

Reference: StemKernel<double,BPMat>::full_dp stem_kernel/stem_kernel.cpp:282-351
and partial_dp with -b (:113-280, alignment_constraints :68-74); defaults of
stem_kernel/main.cpp:46-64 (gap 0.8, stack 1.0, subst 0.5, loop 3, bp_bound 0).
Expected values: the CPU oracle (oracle/sk_oracle.c; parity against the
reference's own output is unpinned).  The synthetic fold's bytes
are pinned by a SHA-256 stored beside the values.

Run:  python tests/golden/make_golden_4d_long.py      (~1 min on 8 cores)
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
    """(x, y, band): |y| = 600 (2 tiles), 1,100 (3 tiles), a banded |y| = 530,
    and |x| = 520 against a short y."""
    s = lambda L, k: ska.random_sequences(1, L, 0x5EED0400 + k)[0]
    return [(s(40, 1), s(600, 2), 0), (s(30, 3), s(1100, 4), 0), (s(60, 5), s(530, 6), 10),
            (s(520, 7), s(45, 8), 0), (s(600, 2), s(40, 1), 0)]


def _cell(c):
    a, b, band = c
    return po.stem4d(a.lower(), ska.fold(a.lower()), b.lower(), ska.fold(b.lower()),
                     float(np.float32(0.8)), 1.0, 0.5, 0.0, 0, 3, band)


def main():
    cs = cases()
    with ProcessPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        vals = list(ex.map(_cell, cs))
    h = hashlib.sha256()
    for a, b, _ in cs:
        for t in (a, b):
            h.update(np.ascontiguousarray(ska.fold(t.lower()), np.float64).tobytes())
    np.savez_compressed(os.path.join(HERE, "long_4d.npz"), x=np.array([c[0] for c in cs]),
                        y=np.array([c[1] for c in cs]), band=np.array([c[2] for c in cs], np.int32),
                        value=np.array(vals), sha=np.array(h.hexdigest()))
    print(vals)


if __name__ == "__main__":
    main()
