"""Compute stub for ``bench.py --cpu-stub tests.bench_stub:compute``: the C
oracle (test infrastructure) in place of the GPU engine, so the N-rank bench
path -- spawned ranks, the cyclic plan's step slices, the all-gather and the
max-over-ranks timing -- runs on a machine without a GPU."""
import numpy as np

_OM = {}


def compute(data, params, x, y):
    import stem_kernel_amd as ska
    from oracle import pyoracle as po

    def om(i):
        if i not in _OM:
            rows = data[i] if isinstance(data[i], list) else [data[i]]
            _OM[i] = po.OMData(rows, [ska.fold(r.replace("-", "")) for r in rows], 0.01)
        return _OM[i]
    return np.array([po.kernel_value(params.kind, om(int(a)), om(int(b)), params) for a, b in zip(x, y)])


def fail_on_rank1(data, params, x, y):
    """Rank 1 fails before its first all-gather; rank 0 would wait there."""
    import os
    if os.environ.get("RANK") == "1":
        raise RuntimeError("injected rank-1 failure")
    return compute(data, params, x, y)
