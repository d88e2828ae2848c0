import sys, time, os
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
def log(*a): print(f"[{time.time()-T0:7.2f}]", *a, flush=True)
T0 = time.time()
import stem_kernel_amd as ska
log("import ok")
seqs = ska.random_sequences(3, 40, 7)
ds = ska.Dataset.from_sequences(seqs)
log("dataset ok", [ds.shape(i) for i in range(3)])
ctx = ska.Context(0)
log("context ok")
ctx.upload(ds)
log("upload ok")
which = sys.argv[1] if len(sys.argv) > 1 else "str"
kern = ska.StringKernel() if which == "str" else ska.SuStemKernel()
v = ctx.pairs(ds, kern, np.array([0], np.int32), np.array([1], np.int32))
log("pairs ok", v, ctx.last_timing())
from oracle import pyoracle as po
om = [po.OMData([s], [ska.fold(s)]) for s in seqs]
log("oracle", po.kernel_value(kern.params.kind, om[0], om[1], kern.params))
