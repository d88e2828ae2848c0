"""String kernel fast path, step by step (development tool)."""
import sys
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples

ctx = ska.Context(0)
kern = ska.StringKernel(gap=0.8, alpha=0.2)
for L in (10, 64, 65, 130):
    seqs = ska.random_sequences(2, L, 0x5EED0C00 + L)
    ds, om = make_examples(seqs)
    print("L", L, "start", flush=True)
    got = ctx.pairs(ds, kern, np.array([0, 1, 0], np.int32), np.array([0, 1, 1], np.int32))
    ref = [po.kernel_value(kern.params.kind, om[a], om[b], kern.params) for a, b in ((0, 0), (1, 1), (0, 1))]
    print("L", L, got, ref, flush=True)
