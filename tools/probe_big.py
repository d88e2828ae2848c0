"""Probe the big-y DAG stem kernel: time and parity of one forced call."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import stem_kernel_amd as ska
from oracle import pyoracle as po

ctx = ska.Context(0)
for L in [int(a) for a in sys.argv[1:]]:
    seqs = ska.random_sequences(2, L, 0x5EED0300 + L)
    ds = ska.Dataset.synthetic(seqs)
    om = [po.OMData([s], [ska.fold(s.lower())], 0.01) for s in seqs]
    ref = po.kernel_value(0, om[0], om[1], ska.SuStemKernel().params)
    for force in ("0", "1"):
        os.environ["SK_FORCE_BIG_Y"] = force
        t = time.perf_counter()
        got = ctx.pairs(ds, ska.SuStemKernel(), [0], [1])[0]
        dt = time.perf_counter() - t
        print(f"L={L} force={force} nl={ds.shape(1)} {dt*1e3:.1f} ms rel={abs(got-ref)/abs(ref):.2e} "
              f"classes={ctx.last_classes()['stem_maxk']}", flush=True)
