"""Quick throughput probe of the stem DP on one GPU (development tool)."""
import sys, time
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import stem_kernel_amd as ska

L = int(sys.argv[1]) if len(sys.argv) > 1 else 200
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
kind = sys.argv[3] if len(sys.argv) > 3 else "stem"
t = time.time()
seqs = ska.random_sequences(N, L, 0x5EED0000 + 2)
ds = ska.Dataset.from_sequences(seqs, th=0.01)
print(f"build {N} examples: {time.time()-t:.2f}s", flush=True)
ctx = ska.Context(0)
ctx.upload(ds)
kern = {"stem": ska.SuStemKernel(), "str": ska.StringKernel(), "ss": ska.SuStemStrKernel(),
        "bpla": ska.BPLAKernel(), "la": ska.BPLAKernel(noBP=True), "stem4d": ska.StemKernel4D(),
        "stem4d_ali": ska.StemKernel4D(ali_bound=0.5, ali_zerop_fixed=True),
        "stem4d_ali0": ska.StemKernel4D(ali_bound=0.5),
        "stem4d_b10": ska.StemKernel4D(band=10)}[kind]
iu = np.triu_indices(N)
x, y = iu[0].astype(np.int32), iu[1].astype(np.int32)
if len(sys.argv) > 4:  # limit the pair count (4-D kernel)
    x, y = x[: int(sys.argv[4])], y[: int(sys.argv[4])]
for rep in range(2):
    t = time.time()
    v = ctx.pairs(ds, kern, x, y)
    dt = time.time() - t
    tm = ctx.last_timing()
    print(f"L={L} N={N} pairs={x.size} wall={dt*1e3:.1f}ms pairs/s={x.size/dt:.0f} "
          f"stem_ms={tm['stem_ms']:.1f} str_ms={tm['string_ms']:.1f} cells={tm['cells']:.3g} "
          f"cells/s={tm['cells']/max(tm['stem_ms'],1e-9)*1e3:.3g}", flush=True)
print("finite", np.all(np.isfinite(v)), "min", v.min(), "max", v.max())
