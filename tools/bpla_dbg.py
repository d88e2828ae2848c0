"""BPLA fast path: per-pair relative error of the grouped (chunked) and the
one-pair-per-wave kernels against the oracle (development tool)."""
import os, sys
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import stem_kernel_amd as ska
from oracle import pyoracle as po
from tests.helpers import make_examples
from tests.test_bpla import _examples

ds, om = make_examples(_examples())
n = len(om)
ctx = ska.Context(0)
kern = ska.BPLAKernel()
x = np.tile(np.arange(n, dtype=np.int32), 24)
y = np.repeat(np.array([0, 11, 12], np.int32), x.size // 3 + 1)[: x.size]
ref = np.array([po.kernel_value(kern.params.kind, om[a], om[b], kern.params) for a, b in zip(x, y)])
for env in ({"SK_BPLA_CHUNK": "1"}, {"SK_BPLA_CHUNK": "4"}, {"SK_BPLA_NO_ITEMS": "1"}):
    os.environ.update(env)
    got = ctx.pairs(ds, kern, x, y)
    for k in env:
        del os.environ[k]
    e = np.abs(got - ref) / np.abs(ref)
    bad = np.argsort(-e)[:6]
    print(env, "max", e.max(), [(int(x[b]), int(y[b]), float(e[b])) for b in bad], flush=True)
print("lens", [ds.shape(i)[4] for i in range(n)])
# determinism: identical pairs within a launch and across launches
for env in ({"SK_BPLA_GENERAL": "1"}, {"SK_BPLA_CHUNK": "4"}, {"SK_BPLA_CHUNK": "1"}):
    os.environ.update(env)
    g1 = ctx.pairs(ds, kern, x, y)
    g2 = ctx.pairs(ds, kern, x, y)
    for k in env:
        del os.environ[k]
    spread = 0.0
    for p in set(zip(x.tolist(), y.tolist())):
        sel = (x == p[0]) & (y == p[1])
        v = g1[sel]
        spread = max(spread, float((v.max() - v.min()) / abs(v).max()))
    e = np.abs(g1 - ref) / np.abs(ref)
    print(env, "runs equal", np.array_equal(g1, g2), "max spread within run", spread, "max err", e.max(),
          "argmax", int(x[e.argmax()]), int(y[e.argmax()]), flush=True)
