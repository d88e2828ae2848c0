"""Throughput probe of the BPLA gradient kernel (development tool)."""
import sys, time
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import stem_kernel_amd as ska
from bench import c4_alignments

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
alns = c4_alignments(N, 190, 210, 4, 0x5EED0003)
ds = ska.Dataset.synthetic_alignments(alns, th=0.01, threads=16)
ctx = ska.Context(0)
iu = np.triu_indices(N)
x, y = iu[0].astype(np.int32), iu[1].astype(np.int32)
for rep in range(2):
    t = time.time()
    v, g = ctx.bpla_gradients(ds, ska.BPLAKernel(), x, y)
    dt = time.time() - t
    print(f"N={N} pairs={x.size} wall={dt*1e3:.1f}ms pairs/s={x.size/dt:.0f} "
          f"kernel_ms={ctx.last_timing()['stem_ms']:.1f} finite={np.all(np.isfinite(g))}", flush=True)
