"""Generate tests/golden/*.npz: seeded inputs (sequences/alignments and their
base-pairing matrices) with the oracle's kernel values.

The reference cannot be built or run here (Boost/ViennaRNA/config.h absent,
see DESIGN.md §Oracle) and ships no fixtures, so these vectors are produced by
the CPU oracle (oracle/sk_oracle.c).  They pin the oracle and the GPU engine
against regressions; the oracle itself is pinned to the reference only for
the alphabet/profile/RIBOSUM pieces (tests/test_oracle_pinning.py).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import stem_kernel_amd as ska  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from tests.helpers import mutate_alignment  # noqa: E402

KINDS = {0: "SuStem", 1: "SiStem", 2: "SuStr", 3: "SiStr", 4: "SuStemStr", 5: "SiStemStr",
         6: "LSuStem", 7: "LSuStemStr"}


def main():
    base = ska.random_sequences(2, 64, 0x5EED0001)
    examples = [[s] for s in ska.random_sequences(5, 72, 0x5EED0001 + 7)]
    examples += [[ska.random_sequences(1, 41, 11)[0]], ["GGGGAAACCCCAUGCGCAAAGCGCAU"],
                 mutate_alignment(base[0], 3, 1), mutate_alignment(base[1], 2, 2)]
    rows_flat, bpp_flat, ex_rows = [], [], []
    for ex in examples:
        ex_rows.append(len(ex))
        for r in ex:
            rows_flat.append(r)
            bpp_flat.append(ska.fold(r.replace("-", "").lower()))
    om = []
    k = 0
    for nr in ex_rows:
        om.append(po.OMData(rows_flat[k:k + nr], bpp_flat[k:k + nr], 0.01))
        k += nr
    n = len(om)
    p = ska.SuStemStrKernel().params  # defaults: also the other kinds' parameters
    vals = {}
    for kind in KINDS:
        m = np.full((n, n), np.nan)
        for i in range(n):
            for j in range(n):
                m[i, j] = po.kernel_value(kind, om[i], om[j], p)
        vals[f"K{kind}"] = m
    naive_seqs = ska.random_sequences(6, 80, 0x5EED0000)  # config C1 shape (L=80)
    naive = np.array([[po.naive_string(a, b, 0.8) for b in naive_seqs] for a in naive_seqs])
    shapes = np.array([[v.size for v in (d["first"], d["edge_to"], d["bp_code"], d["roots"])]
                       for d in (o.dag() for o in om)])
    np.savez_compressed(
        os.path.join(HERE, "lite_small.npz"),
        rows=np.array(rows_flat), ex_rows=np.array(ex_rows),
        bpp=np.array(np.concatenate(bpp_flat)), bpp_len=np.array([b.size for b in bpp_flat]),
        shapes=shapes, naive_seqs=np.array(naive_seqs), naive=naive, **vals)
    meta = {"kinds": KINDS, "th": 0.01,
            "params": {f: getattr(p, f) for f, _ in type(p)._fields_}}
    json.dump(meta, open(os.path.join(HERE, "lite_small.json"), "w"), indent=1)
    print("wrote", os.path.join(HERE, "lite_small.npz"), n, "examples")


if __name__ == "__main__":
    main()
