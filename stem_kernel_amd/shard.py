"""Multi-GPU Gram sharding (one process per GPU).

Every Gram cell K(i,j), i <= j, is independent (common/kernel_matrix.cpp:44-55).
The plan is the reference MPI Gram's: upper-triangle cell k (row-major) goes
to rank k % P (CalcTrainMatrix::operator(), common/kernel_matrix.cpp:210-224),
which gives every rank the same cost mix.  Each rank computes its cells into
an equal-sized buffer, ONE all-gather joins the buffers on every rank, and
every rank assembles the mirrored, normalised matrix (the reference's
Ssend/Recv to rank 0 and replayed scatter, :225-261, 495-527).  Plan and
assembly are the C ABI's (sk_shard_cells / sk_shard_assemble,
csrc/host/shard.cpp), so a C++ host and this module produce the same bits.

Two transports:

* ``gram_rccl`` -- the product path: the engine's own RCCL communicator
  (sk_comm_init), its cells written into a device buffer and all-gathered by
  sk_gram_sharded inside the library; torch.distributed only hands the
  128-byte RCCL id from rank 0 to the others.
* ``distributed_gram`` -- any torch.distributed backend (gloo on CPU for the
  multi-process tests, nccl = RCCL on GPUs) with a caller-supplied compute.

The plan is a pure function of (n, world) and values depend only on the pair,
so the N-GPU Gram is bit-identical to the 1-GPU Gram.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Tuple

import numpy as np

from ._lib import check, lib


def shard_count(n: int, world: int, rank: int) -> int:
    """Cells of `rank` (sk_shard_count)."""
    return int(lib().sk_shard_count(n, rank, world))


def rank_pairs(n: int, world: int, rank: int) -> Tuple[np.ndarray, np.ndarray]:
    """Upper-triangle cells (i <= j) of `rank`, in cell order (sk_shard_cells)."""
    m = shard_count(n, world, rank)
    x = np.zeros(max(m, 1), np.int32)
    y = np.zeros(max(m, 1), np.int32)
    check(lib().sk_shard_cells(n, rank, world, x.ctypes.data_as(C.POINTER(C.c_int32)),
                               y.ctypes.data_as(C.POINTER(C.c_int32))))
    return x[:m], y[:m]


def max_pairs(n: int, world: int) -> int:
    """Equal buffer size of the all-gather: rank 0 has the most cells."""
    return max(shard_count(n, world, 0), 1)


def assemble(parts, n: int, world: int, normalize: bool = False) -> np.ndarray:
    """Scatter the ranks' buffers (parts[r][:count_r]) into the mirrored n x n
    matrix and normalise as KernelMatrix::calculate does
    (kernel_matrix.cpp:560-571), through sk_shard_assemble."""
    per = max_pairs(n, world)
    g = np.zeros((world, per), np.float64)
    for r in range(world):
        v = np.asarray(parts[r], dtype=np.float64).ravel()
        c = shard_count(n, world, r)
        g[r, :c] = v[:c]
    out = np.zeros((n, n), np.float64)
    check(lib().sk_shard_assemble(n, world, g.ctypes.data_as(C.POINTER(C.c_double)), per,
                                  int(normalize), out.ctypes.data_as(C.POINTER(C.c_double))))
    return out


def distributed_gram(compute: Callable[[np.ndarray, np.ndarray], "object"], n: int,
                     normalize: bool = False, group=None, device=None) -> np.ndarray:
    """Gram over a torch.distributed group: compute(x, y) returns this rank's
    values (a torch tensor on `device`, or a host array), then one
    all_gather_into_tensor of equal-sized buffers."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    x, y = rank_pairs(n, world, rank)
    cap = max_pairs(n, world)
    vals = compute(x, y)
    if not torch.is_tensor(vals):
        vals = torch.as_tensor(np.asarray(vals, dtype=np.float64))
    dev = vals.device if device is None else device
    buf = torch.zeros(cap, dtype=torch.float64, device=dev)
    buf[: x.size] = vals.to(dev)
    out = torch.empty(cap * world, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    return assemble(out.cpu().numpy().reshape(world, cap), n, world, normalize)


def build_split(build: Callable[[int, int], "object"], n: int, group=None):
    """Build a dataset of n examples in rank shares: rank r of the group
    builds examples [n*r/N, n*(r+1)/N) with build(first, last) (a Dataset of
    those examples, in order), the shares are gathered as bytes
    (Dataset.export / sk_dataset_export) and every rank appends them in rank
    order -- the same examples, bit for bit, as one rank building all n, so
    the packed arrays are too (tests/test_distributed.py).  The reference's
    MPI Gram has every rank read and build every example
    (common/kernel_matrix.cpp:186-261)."""
    import torch.distributed as dist

    from .kernel_matrix import Dataset

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = n * rank // world, n * (rank + 1) // world
    part = build(lo, hi)
    if len(part) != hi - lo:
        raise ValueError(f"build({lo}, {hi}) returned {len(part)} examples")
    parts = [None] * world
    dist.all_gather_object(parts, part.export(), group=group)
    out = Dataset()
    for b in parts:
        out.import_bytes(b)
    return out


def rccl_init(ctx, group=None) -> None:
    """Give `ctx` its own RCCL communicator over the ranks of a
    torch.distributed group: rank 0 draws the id (sk_comm_unique_id), the
    group broadcasts the 128 bytes, every rank calls sk_comm_init."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    obj = [None]
    if rank == 0:
        buf = C.create_string_buffer(128)
        check(lib().sk_comm_unique_id(buf, 128))
        obj[0] = buf.raw
    dist.broadcast_object_list(obj, src=0, group=group)
    ctx.comm_init(obj[0], rank, world)


def gram_rccl(ctx, ds, kernel, normalize: bool = False) -> np.ndarray:
    """The sharded Gram through the engine (sk_gram_sharded): every rank
    passes the same dataset and gets the whole matrix."""
    return ctx.gram_sharded(ds, kernel, normalize)


def gpu_compute(ctx, ds, kernel, device):
    """compute() for distributed_gram: the HIP engine writing straight into a
    device buffer (no host round trip before the all-gather)."""
    import torch

    def f(x, y):
        out = torch.empty(max(x.size, 1), dtype=torch.float64, device=device)
        if x.size:
            ctx.pairs_device(ds, kernel, x, y, out.data_ptr())
        return out[: x.size]

    return f


def assemble_gradients(x, y, val, grad, n: int, normalize: bool = False):
    """The bpla_optimizer's Gram and gradient matrices from per-pair values
    and d/d(alpha, beta, gap, ext) of the cells (x[k] <= y[k]) covering the
    upper triangle: CalcMatrix (bpla_optimizer.cpp:52-126, mirrored) or, with
    normalize, CalcMatrixN (:128-255: K/sqrt(K_ii K_jj), its derivative,
    diagonal 1 and 0).  Returns (K[n, n], G[4, n, n])."""
    x = np.asarray(x)
    y = np.asarray(y)
    val = np.asarray(val, dtype=np.float64)
    grad = np.asarray(grad, dtype=np.float64).reshape(-1, 4)
    K = np.zeros((n, n))
    G = np.zeros((4, n, n))
    if not normalize:
        K[x, y] = val
        K[y, x] = val
        for l in range(4):
            G[l, x, y] = grad[:, l]
            G[l, y, x] = grad[:, l]
        return K, G
    d = x == y
    dk = np.zeros(n)
    dg = np.zeros((4, n))
    dk[x[d]] = val[d]
    dg[:, x[d]] = grad[d].T
    off = ~d
    i, j = x[off], y[off]
    sq = np.sqrt(dk[i] * dk[j])
    k = val[off] / sq
    K[i, j] = K[j, i] = k
    np.fill_diagonal(K, 1.0)
    for l in range(4):
        g = grad[off, l] / sq - k / 2 * (dg[l, i] / dk[i] + dg[l, j] / dk[j])
        G[l, i, j] = G[l, j, i] = g
    return K, G


def distributed_gradient_gram(compute, n: int, normalize: bool = False, group=None, device=None):
    """bpla_optimizer's Gram + gradient matrices over the process group (the
    reference Bcasts every rank's cells over MPI, bpla_optimizer.cpp:62-104):
    compute(x, y) returns (values[k], grads[k, 4]) for this rank's cells of
    the cyclic plan, then ONE all_gather_into_tensor of equal-sized (cap, 5)
    buffers; every rank assembles the same matrices."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    x, y = rank_pairs(n, world, rank)
    cap = max_pairs(n, world)
    val, grad = compute(x, y)
    v = torch.as_tensor(np.asarray(val, dtype=np.float64)) if not torch.is_tensor(val) else val
    g = torch.as_tensor(np.asarray(grad, dtype=np.float64)) if not torch.is_tensor(grad) else grad
    dev = v.device if device is None else device
    buf = torch.zeros((cap, 5), dtype=torch.float64, device=dev)
    buf[: x.size, 0] = v.to(dev)
    buf[: x.size, 1:] = g.reshape(-1, 4).to(dev)
    out = torch.empty((world * cap, 5), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    parts = out.cpu().numpy().reshape(world, cap, 5)
    xs, ys, vs, gs = [], [], [], []
    for r in range(world):
        rx, ry = rank_pairs(n, world, r)
        xs.append(rx)
        ys.append(ry)
        vs.append(parts[r, : rx.size, 0])
        gs.append(parts[r, : rx.size, 1:])
    return assemble_gradients(np.concatenate(xs), np.concatenate(ys), np.concatenate(vs),
                              np.concatenate(gs), n, normalize)
