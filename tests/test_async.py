"""Asynchronous compute calls (sk_set_async): results equal the synchronous
calls' bit for bit, host inputs may be freed as soon as a call returns
(pinned staging), and sk_sync_timing sums the timings of every call since
the previous one.  The bench runs its steps this way (bench.py GpuEngine)."""
import gc

import numpy as np
import pytest

import stem_kernel_amd as ska


@pytest.fixture(scope="module")
def sets():
    seqs = ska.random_sequences(24, 90, 0x5EED0A51)
    ds = ska.Dataset.synthetic(seqs, th=0.01, threads=4)
    alns = [[s, s[::-1]] for s in ska.random_sequences(16, 70, 0x5EED0A52)]
    da = ska.Dataset.synthetic_alignments(alns, th=0.01, threads=4)
    return ds, da


def _pairs(n, seed, count):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, n, count).astype(np.int32)
    y = rng.integers(0, n, count).astype(np.int32)
    return x, y


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["lss", "stem", "bpla"])
def test_async_calls_equal_sync(sets, which):
    import torch
    ds_s, ds_a = sets
    ds = ds_a if which == "bpla" else ds_s
    kern = {"lss": ska.LSuStemStrKernel(), "stem": ska.SuStemKernel(), "bpla": ska.BPLAKernel()}[which]
    ctx = ska.Context(0)
    try:
        calls = [_pairs(len(ds), 11 + k, 150 + 37 * k) for k in range(6)]
        ref = [ctx.pairs(ds, kern, x, y) for x, y in calls]
        sync_cells = []
        for x, y in calls:
            ctx.pairs(ds, kern, x, y)
            sync_cells.append(ctx.last_timing()["cells"])
        ctx.set_async(True)
        outs = []
        for x, y in calls:  # more calls than the ring of timing sets (4)
            o = torch.full((x.size,), float("nan"), dtype=torch.float64, device="cuda:0")
            xa, ya = x.copy(), y.copy()
            ctx.pairs_device(ds, kern, xa, ya, o.data_ptr())
            del xa, ya  # the call's host inputs die at once: staged
            gc.collect()
            outs.append(o)
        torch.cuda.synchronize()
        ctx.sync_timing()
        tot = ctx.last_timing()
        assert tot["cells"] == pytest.approx(sum(sync_cells), rel=1e-12)
        assert tot["stem_ms"] > 0.0 and ctx.last_launch_ms()["launches"] >= len(calls)
        for o, r in zip(outs, ref):
            assert np.array_equal(o.cpu().numpy(), r)
        # host-result calls stay correct in async mode (stream-ordered copy)
        x, y = calls[0]
        assert np.array_equal(ctx.pairs(ds, kern, x, y), ref[0])
        ctx.set_async(False)
        assert np.array_equal(ctx.pairs(ds, kern, x, y), ref[0])
    finally:
        ctx.close()
