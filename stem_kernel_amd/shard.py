"""Multi-GPU Gram sharding (one process per GPU, torch.distributed / RCCL).

Every Gram cell K(i,j), i <= j, is independent (common/kernel_matrix.cpp:44-55),
so the upper triangle is partitioned with no data-path collective: rank g
takes the row blocks g and 2P-1-g of 2P equal row blocks (folding equalises
the triangle area), computes its cells, and ONE all-gather of equal-sized
buffers assembles the matrix on every rank.  The reference dealt cells
cyclically to MPI ranks and gathered to rank 0 point-to-point
(common/kernel_matrix.cpp:186-261, 495-527).

The partition is a pure function of (n, world), so the N-GPU Gram is
bit-identical to the 1-GPU Gram.
"""
from __future__ import annotations

import math
from typing import Callable, Tuple

import numpy as np


def folded_row_blocks(n: int, world: int, rank: int) -> np.ndarray:
    """Rows owned by `rank`: blocks rank and 2*world-1-rank of 2*world."""
    nb = 2 * world
    edges = [round(n * b / nb) for b in range(nb + 1)]
    rows = []
    for b in (rank, nb - 1 - rank):
        rows.extend(range(edges[b], edges[b + 1]))
    return np.array(sorted(set(rows)), dtype=np.int32)


def rank_pairs(n: int, world: int, rank: int) -> Tuple[np.ndarray, np.ndarray]:
    """Upper-triangle cells (i <= j) of the rows `rank` owns, row-major."""
    rows = folded_row_blocks(n, world, rank)
    xs, ys = [], []
    for i in rows:
        xs.append(np.full(n - i, i, np.int32))
        ys.append(np.arange(i, n, dtype=np.int32))
    if not xs:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    return np.concatenate(xs), np.concatenate(ys)


def max_pairs(n: int, world: int) -> int:
    return max(rank_pairs(n, world, r)[0].size for r in range(world))


def assemble(parts, n: int, world: int, normalize: bool = False) -> np.ndarray:
    """Scatter every rank's values into the mirrored n x n matrix and
    normalise as KernelMatrix::calculate does (kernel_matrix.cpp:560-571)."""
    m = np.zeros((n, n), dtype=np.float64)
    for r in range(world):
        x, y = rank_pairs(n, world, r)
        v = np.asarray(parts[r])[: x.size]
        m[x, y] = v
        m[y, x] = v
    if normalize and n > 0:
        out = m.copy()
        for i in range(n - 1):
            for j in range(i + 1, n):
                out[i, j] = m[i, j] / math.sqrt(m[i, i] * m[j, j])
                out[j, i] = out[i, j]
        np.fill_diagonal(out, 1.0)
        m = out
    return m


def distributed_gram(compute: Callable[[np.ndarray, np.ndarray], "object"], n: int,
                     normalize: bool = False, group=None, device=None) -> np.ndarray:
    """Gram over the default process group: compute(x, y) returns this rank's
    values (a torch tensor on `device`, or host array for CPU/gloo), then one
    all_gather_into_tensor of padded, equal-sized buffers."""
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
    parts = out.cpu().numpy().reshape(world, cap)
    return assemble(parts, n, world, normalize)


def gpu_compute(ctx, ds, kernel, device):
    """compute() for distributed_gram: the HIP engine writing straight into a
    device buffer (no host round trip before the RCCL all-gather)."""
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
    the folded row-block plan, then ONE all_gather_into_tensor of equal-sized
    (cap, 5) buffers; every rank assembles the same matrices."""
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
