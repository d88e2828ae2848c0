"""DAG sizes of the NS inputs under the synthetic Nussinov-Boltzmann bpp
stand-in vs the engine's McCaskill fold (development tool)."""
import sys
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import stem_kernel_amd as ska

seqs = ska.random_sequences(4096, 200, 0x5EED0000 + 2)[:256]
ctx = ska.Context(0)
syn = ska.Dataset.synthetic(seqs, th=0.01)
fol = ska.Dataset.folded(ctx, seqs, th=0.01)
for name, ds in (("synthetic", syn), ("mccaskill", fol)):
    sh = np.array([ds.shape(i) for i in range(len(seqs))], dtype=np.float64)
    print(f"{name:10s} nodes {sh[:,0].mean():.0f} edges {sh[:,1].mean():.0f} bpfreq {sh[:,2].mean():.0f}", flush=True)
kern = ska.SuStemStrKernel()
x, y = np.triu_indices(len(seqs))
for name, ds in (("synthetic", syn), ("mccaskill", fol)):
    ctx.pairs(ds, kern, x.astype(np.int32), y.astype(np.int32))
    import time
    t = time.time()
    ctx.pairs(ds, kern, x.astype(np.int32), y.astype(np.int32))
    dt = time.time() - t
    print(f"{name:10s} {x.size / dt:.0f} pairs/s (256-example Gram)", flush=True)
