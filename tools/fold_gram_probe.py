"""Steady-state Gram throughput on McCaskill-folded inputs (development tool):
N sequences of length L, SuStemStr, with the launched classes."""
import sys, time
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import stem_kernel_amd as ska

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
L = int(sys.argv[2]) if len(sys.argv) > 2 else 200
seqs = ska.random_sequences(N, L, 0x5EED0000 + 2)
ctx = ska.Context(0)
t = time.time()
ds = ska.Dataset.folded(ctx, seqs, th=0.01)
print(f"fold+build {time.time() - t:.2f}s", flush=True)
sh = np.array([ds.shape(i) for i in range(N)], dtype=np.float64)
print(f"nodes {sh[:,0].mean():.0f} (max {sh[:,0].max():.0f}) edges {sh[:,1].mean():.0f}", flush=True)
x, y = np.triu_indices(N)
x, y = x.astype(np.int32), y.astype(np.int32)
for kern in (ska.SuStemStrKernel(), ska.SuStemKernel(), ska.StringKernel()):
    ctx.pairs(ds, kern, x[:100000], y[:100000])
    t = time.time()
    ctx.pairs(ds, kern, x, y)
    dt = time.time() - t
    tm = ctx.last_timing()
    print(f"{type(kern).__name__}: {x.size / dt:.0f} pairs/s wall, stem {tm['stem_ms']:.1f} ms, "
          f"string {tm['string_ms']:.1f} ms, launches {tm['launches']}, classes {ctx.last_classes()}", flush=True)
