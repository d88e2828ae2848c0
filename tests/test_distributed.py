"""Multi-process path on CPU: world_size-2 gloo over 127.0.0.1.

The shard plan (the reference MPI Gram's cyclic cell deal, sk_shard_cells)
must cover the upper triangle exactly once, and the gathered, mirrored,
normalised Gram must equal the single-process one bit for bit (the compute
function is the oracle here; on GPUs it is the engine: sk_gram_sharded over
its own RCCL communicator, or shard.gpu_compute).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from stem_kernel_amd import shard


@pytest.mark.parametrize("n,world", [(1, 2), (7, 2), (10, 3), (33, 4), (64, 8)])
def test_plan_covers_triangle_once(n, world):
    seen = np.zeros((n, n), int)
    for r in range(world):
        x, y = shard.rank_pairs(n, world, r)
        assert np.all(x <= y)
        np.add.at(seen, (x, y), 1)
    assert np.array_equal(seen, np.triu(np.ones((n, n), int)))
    sizes = [shard.rank_pairs(n, world, r)[0].size for r in range(world)]
    assert max(sizes) - min(sizes) <= 1  # cyclic deal: equal shares
    # the reference's order: cell k of the row-major triangle to rank k % P
    # (common/kernel_matrix.cpp:210-224)
    iu, ju = np.triu_indices(n)
    for r in range(world):
        x, y = shard.rank_pairs(n, world, r)
        assert np.array_equal(x, iu[r::world]) and np.array_equal(y, ju[r::world])


def test_assemble_matches_reference_normalisation():
    """sk_shard_assemble (threaded) against a literal restatement of
    kernel_matrix.cpp:560-571, bit for bit, at a size where the host threads
    split the rows."""
    import math
    rng = np.random.default_rng(3)
    n, world = 600, 3
    iu, ju = np.triu_indices(n)
    vals = rng.uniform(0.5, 2.0, iu.size)
    parts = [vals[r::world] for r in range(world)]
    got = shard.assemble(parts, n, world, normalize=True)
    m = np.zeros((n, n))
    m[iu, ju] = vals
    m[ju, iu] = vals
    ref = m.copy()
    for i in range(0, n - 1, 37):  # sampled rows of the reference's loop
        for j in range(i + 1, n):
            ref[i, j] = m[i, j] / math.sqrt(m[i, i] * m[j, j])
        assert np.array_equal(got[i, i + 1:], ref[i, i + 1:])
    assert np.all(np.diag(got) == 1.0) and np.array_equal(got, got.T)
    raw = shard.assemble(parts, n, world, normalize=False)
    assert np.array_equal(raw, m)


def test_assemble_n8192_under_a_second():
    import time
    n, world = 8192, 8
    per = shard.max_pairs(n, world)
    parts = [np.ones(per) for _ in range(world)]
    t = time.perf_counter()
    out = shard.assemble(parts, n, world, normalize=True)
    assert time.perf_counter() - t < 1.0 * max(1, 8 // (os.cpu_count() or 8))
    assert out[0, 1] == 1.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    seqs = ska.random_sequences(7, 50, 0x5EED0004)
    om = [po.OMData([s], [ska.fold(s)], 0.01) for s in seqs]
    p = ska.SuStemStrKernel().params

    def compute(x, y):
        return np.array([po.kernel_value(p.kind, om[a], om[b], p) for a, b in zip(x, y)])

    g = shard.distributed_gram(compute, len(seqs), normalize=True)
    dist.destroy_process_group()
    q.put((rank, g))


def test_gloo_world2_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    seqs = ska.random_sequences(7, 50, 0x5EED0004)
    om = [po.OMData([s], [ska.fold(s)], 0.01) for s in seqs]
    p = ska.SuStemStrKernel().params
    n = len(seqs)
    raw = np.zeros((n, n))
    for i in range(n):
        for j in range(i, n):
            raw[i, j] = raw[j, i] = po.kernel_value(p.kind, om[i], om[j], p)
    ref = shard.assemble([raw[np.triu_indices(n)]], n, 1, normalize=True)
    assert np.array_equal(res[0], res[1])
    assert np.array_equal(res[0], ref)


def _split_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import stem_kernel_amd as ska
    seqs = ska.random_sequences(11, 80, 0x5EED0013)
    ds = shard.build_split(lambda lo, hi: ska.Dataset.synthetic(seqs[lo:hi]), len(seqs))
    dist.destroy_process_group()
    q.put((rank, len(ds), ds.pack_digest()))


def test_gloo_world2_split_build_packs_as_one_rank():
    """shard.build_split: each rank builds its share of the examples, the
    shares are gathered as bytes, and every rank's dataset packs to the same
    arrays as one process building all of them (verdict r05 item 5)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (n, d)) for r, n, d in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    import stem_kernel_amd as ska
    seqs = ska.random_sequences(11, 80, 0x5EED0013)
    whole = ska.Dataset.synthetic(seqs)
    assert res[0] == res[1] == (len(seqs), whole.pack_digest())


@pytest.mark.gpu
def test_rccl_world1_matches_gram_bit_for_bit(gpu_ctx):
    """Both RCCL paths at world 1 -- the engine's own communicator
    (sk_gram_sharded) and torch's nccl backend around gpu_compute -- give
    sk_gram's bits."""
    import torch
    import torch.distributed as dist
    import stem_kernel_amd as ska

    seqs = ska.random_sequences(9, 70, 0x5EED0005)
    ds = ska.Dataset.synthetic(seqs, th=0.01, threads=4)
    kern = ska.SuStemStrKernel()
    ref = gpu_ctx.gram(ds, kern, normalize=True)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    try:
        g = shard.distributed_gram(shard.gpu_compute(gpu_ctx, ds, kern, dev), len(seqs),
                                   normalize=True)
        shard.rccl_init(gpu_ctx)
        g2 = shard.gram_rccl(gpu_ctx, ds, kern, normalize=True)
    finally:
        dist.destroy_process_group()
    assert np.array_equal(g, ref)
    assert np.array_equal(g2, ref)


@pytest.mark.gpu
def test_pair_values_independent_of_batch(gpu_ctx):
    """A cell's value depends only on its pair, not on which other cells share
    the launch or their order -- what makes the N-GPU Gram equal the 1-GPU
    one bit for bit."""
    import stem_kernel_amd as ska

    seqs = ska.random_sequences(12, 200, 0x5EED0002)
    ds = ska.Dataset.synthetic(seqs, th=0.01, threads=4)
    kern = ska.SuStemStrKernel()
    iu, ju = (a.astype(np.int32) for a in np.triu_indices(len(seqs)))
    full = gpu_ctx.pairs(ds, kern, iu, ju)
    perm = np.random.default_rng(1).permutation(iu.size)
    shuf = gpu_ctx.pairs(ds, kern, iu[perm], ju[perm])
    assert np.array_equal(shuf, full[perm])
    for r in range(3):
        part = gpu_ctx.pairs(ds, kern, iu[r::3], ju[r::3])
        assert np.array_equal(part, full[r::3])


def _grad_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    seqs = ska.random_sequences(6, 30, 0x5EED0006)
    om = [po.OMData([s], [ska.fold(s)], 0.01) for s in seqs]
    p = ska.BPLAKernel().params
    t = np.array(list(p.score_table))

    def compute(x, y):
        r = [po.bpla_gradients(om[a], om[b], p.alpha, p.beta, p.gap, p.ext, t) for a, b in zip(x, y)]
        return np.array([v for v, _, _ in r]), np.array([d for _, d, _ in r]).reshape(-1, 4)

    K, G = shard.distributed_gradient_gram(compute, len(seqs), normalize=True)
    dist.destroy_process_group()
    q.put((rank, (K, G)))


def test_gloo_world2_gradient_gram_matches_single_process():
    """bpla_optimizer's Gram + gradient matrices (f4) over two gloo ranks equal
    the single-process assembly of the same cells, bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    seqs = ska.random_sequences(6, 30, 0x5EED0006)
    om = [po.OMData([s], [ska.fold(s)], 0.01) for s in seqs]
    p = ska.BPLAKernel().params
    t = np.array(list(p.score_table))
    n = len(seqs)
    x, y = (a.astype(np.int32) for a in np.triu_indices(n))
    r = [po.bpla_gradients(om[a], om[b], p.alpha, p.beta, p.gap, p.ext, t) for a, b in zip(x, y)]
    K, G = shard.assemble_gradients(x, y, [v for v, _, _ in r], [d for _, d, _ in r], n, True)
    for rank in (0, 1):
        assert np.array_equal(res[rank][0], K) and np.array_equal(res[rank][1], G)
    assert np.allclose(np.diag(K), 1.0) and np.all(G[:, np.arange(n), np.arange(n)] == 0.0)


def _bench(args, timeout=300):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, cwd=root, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints ONE line
    return json.loads(lines[0])


@pytest.mark.parametrize("config,n,length", [("ns", 10, 40), ("c4", 6, 30)])
def test_bench_spawns_its_own_ranks(config, n, length):
    """`bench.py --gpus 2` with no launcher starts two worker ranks itself
    (gloo here, through the CPU compute stub), runs the cyclic plan's step
    slices, all-gathers them and reports the whole job; the gathered slices
    of every rank are checked against the stub inside the run."""
    line = _bench(["--gpus", "2", "--config", config, "--n", str(n), "--length", str(length),
                   "--steps", "2", "--warmup", "1", "--cpu-stub", "tests.bench_stub:compute"])
    assert line["n_gpus"] == 2 and line["steps"] == 2
    assert line["stub_checked_pairs"] > 0
    assert line["value"] > 0 and line["roofline"] is None


def test_bench_rank_failure_stops_the_job():
    """A failing rank ends the whole job with its status (its peer is stopped
    instead of waiting in a collective forever)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--config", "ns",
                        "--n", "6", "--length", "30", "--cpu-stub", "tests.bench_stub:fail_on_rank1"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "injected rank-1 failure" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_plan_with_gpu_values_matches_gram(gpu_ctx, world):
    """sk_gram_sharded's world > 1 data path on one GPU: every rank's cells
    of the cyclic plan computed by the engine (sk_pairs, as sk_gram_sharded's
    sk_pairs_device does), padded to the all-gather's equal buffers and
    unscattered by sk_shard_assemble, equal sk_gram bit for bit -- raw and
    normalised, with n(n+1)/2 not a multiple of the world size."""
    import stem_kernel_amd as ska

    n = 11  # 66 cells: 66 % 4 != 0, 66 % 8 != 0; world 3 divides it
    seqs = ska.random_sequences(n, 90, 0x5EED0007)
    ds = ska.Dataset.synthetic(seqs, th=0.01, threads=4)
    kern = ska.SuStemStrKernel()
    for normalize in (False, True):
        ref = gpu_ctx.gram(ds, kern, normalize=normalize)
        parts = []
        for r in range(world):
            x, y = shard.rank_pairs(n, world, r)
            parts.append(gpu_ctx.pairs(ds, kern, x, y))
        got = shard.assemble(parts, n, world, normalize=normalize)
        assert np.array_equal(got, ref)
