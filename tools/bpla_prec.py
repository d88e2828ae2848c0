"""Max relative error of the BPLA kernels against the C4 oracle fixture
(tests/golden/large_bpla.npz) -- run once with SK_BPLA_GENERAL=1 (general
kernel only) and once without (dyadic fast path)."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
import stem_kernel_amd as ska  # noqa: E402

B = np.load("tests/golden/large_bpla.npz")
rows = [str(r) for r in B["rows"]]
alns = [rows[4 * k:4 * k + 4] for k in range(len(rows) // 4)]
ds = ska.Dataset.synthetic_alignments(alns)
ctx = ska.Context(0)
n = len(alns)
x, y = (a.ravel() for a in np.meshgrid(np.arange(n), np.arange(n), indexing="ij"))
mode = "general" if os.environ.get("SK_BPLA_GENERAL") else "default"
for kind, (nobp, sw) in zip((9, 10, 11, 12), [(False, False), (True, False), (False, True), (True, True)]):
    got = ctx.pairs(ds, ska.BPLAKernel(noBP=nobp, SW=sw), x, y).reshape(n, n)
    ref = B[f"K{kind}"]
    print(mode, kind, float(np.max(np.abs(got - ref) / np.abs(ref))), flush=True)
