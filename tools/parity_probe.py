"""Observed GPU-vs-oracle error per kernel kind on single sequences and on
alignments with gaps (development tool; the tests assert 1e-6)."""
import sys
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples, mutate_alignment

base = ska.random_sequences(4, 80, 0x5EED0F00)
sets = {
    "single": ska.random_sequences(6, 80, 0x5EED0F01),
    "alignments": [mutate_alignment(base[0], 3, 1), mutate_alignment(base[1], 4, 2),
                   mutate_alignment(base[2], 2, 3), [base[3]]],
}
kernels = {"SuStem": ska.SuStemKernel(), "SiStem": ska.SiStemKernel(),
           "String": ska.StringKernel(gap=0.8, alpha=0.2), "SuStemStr": ska.SuStemStrKernel(),
           "LSuStemStr": ska.LSuStemStrKernel(), "BPLA": ska.BPLAKernel(),
           "BPLA-SW": ska.BPLAKernel(SW=True), "LA": ska.BPLAKernel(noBP=True)}
ctx = ska.Context(0)
for sname, items in sets.items():
    ds, om = make_examples(items)
    n = len(items)
    for kname, kern in kernels.items():
        got = ctx.gram(ds, kern)
        ref = np.array([[po.kernel_value(kern.params.kind, om[i], om[j], kern.params) for j in range(n)]
                        for i in range(n)])
        up = np.triu_indices(n)
        e = np.abs(got[up] - ref[up]) / np.maximum(np.abs(ref[up]), 1e-300)
        print(f"{sname:10s} {kname:10s} max rel err {e.max():.3e}", flush=True)
