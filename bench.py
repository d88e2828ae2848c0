#!/usr/bin/env python3
"""Benchmark of the stem-kernel Gram engine on MI355X.

Default workload (BASELINE.json north_star / metric, ``--config ns``): the
4096 x 4096 Gram matrix of SuStemStrKernel (== StemStrKernel of
stem_kernel_lite/ss_kernel.h: DAG stem kernel + profile string kernel,
default parameters of stem_kernel_lite/main.cpp:103-149) over synthetic RNA
sequences of L = 200 nt (splitmix64 sequences, Nussinov-Boltzmann
base-pairing probabilities, --basepair 0.01).  Units are Gram cells K(i,j),
i <= j, exactly the cells the reference evaluates
(common/kernel_matrix.cpp:44-55): 8,390,656 sequence pairs.

A *step* is one slice of that upper triangle, 1/S of its cells per GPU.  The
product's sharded Gram (sk_gram_sharded, the reference MPI Gram's cyclic plan,
kernel_matrix.cpp:210-224) gives rank r of N the cells k % N == r (k =
row-major index of cell (i, j), i <= j), and every slice is a subset of that
plan, so over S/N steps a rank computes exactly its share of the shipped
Gram.  DAG kernels (ns, c2, c5): the columns j (the y examples) are folded in
pairs (j, n-1-j: n+1 cells per pair) and the pairs dealt round-robin to S/N
column groups of equal cost; step t is column group t, rank r taking its
cells k % N == r -- each y keeps the same share of its column as in the full
Gram (about (j+1)/N pairs), so a step has the full Gram's composition.  Other
kernels: cell k is in slice k % S and rank r computes slice (t*N + r).  Per-GPU
work is fixed, so scaling is weak; the ranks all-gather the step's Gram
entries with the engine's own RCCL communicator (sk_comm_allgather).  --full
times one call of the product path itself: sk_gram_sharded over all N ranks
(cells, all-gather, host assembly of the whole mirrored matrix).

Other SURVEY.md §8 configurations (--config): c2 ss_kernel 256 x L150,
c3 4-D stem kernel 1024 x L200, c4 BPLA 2048 alignments L~200, c5 DAG stem
8192 x L300.  They print the same JSON line for their own kernel.

Timed region: inputs (packed examples) already resident in HBM; each step =
the kernel launches for the slice + the all-gather.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
PEAK_FP64_TFS = 78.6    # FP64 vector

# name -> kernel, n examples, length, slices, config id (seed 0x5EED0000+id)
CONFIGS = {
    "ns": dict(kernel="ss", n=4096, L=200, slices=48, cid=2, cpu_pairs=12288),
    "c2": dict(kernel="ss", n=256, L=150, slices=4, cid=1, cpu_pairs=12288),
    "c3": dict(kernel="stem4d", n=1024, L=200, slices=2050, cid=2, cpu_pairs=32),
    "c4": dict(kernel="bpla", n=2048, L=(190, 210), rows=4, slices=16, cid=3, cpu_pairs=196608),
    "c5": dict(kernel="stem", n=8192, L=300, slices=128, cid=4, cpu_pairs=4096),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=None, help="number of examples")
    ap.add_argument("--length", type=int, default=None)
    ap.add_argument("--slices", type=int, default=None)
    ap.add_argument("--full", action="store_true", help="time every slice (whole Gram)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-pairs", type=int, default=None, help="pairs in the CPU sample")
    ap.add_argument("--pmc-json", default=None)
    return ap.parse_args()


# ------------------------------------------------------------------ inputs
def c4_alignments(n, lo, hi, rows, seed):
    """SURVEY.md §8d C4 generator: per alignment a seed sequence of length
    U[lo,hi], rows with 10% point substitutions and 5% gap characters."""
    import stem_kernel_amd as ska
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, size=n)
    base = ska.random_sequences(n, hi, seed)
    out = []
    acgu = np.frombuffer(b"ACGU", np.uint8)
    for k in range(n):
        s = np.frombuffer(base[k][: lens[k]].encode(), np.uint8)
        aln = []
        for _ in range(rows):
            u = rng.random(s.size)
            r = s.copy()
            sub = (u >= 0.05) & (u < 0.15)
            r[sub] = acgu[rng.integers(0, 4, size=int(sub.sum()))]
            r[u < 0.05] = ord("-")
            aln.append(r.tobytes().decode())
        out.append(aln)
    return out


def build_inputs(cfg, a):
    import stem_kernel_amd as ska
    seed = 0x5EED0000 + cfg["cid"]
    threads = host_threads()
    if cfg["kernel"] == "bpla":
        alns = c4_alignments(a.n, cfg["L"][0], cfg["L"][1], cfg["rows"], seed)
        return alns, ska.Dataset.synthetic_alignments(alns, th=0.01, threads=threads)
    seqs = ska.random_sequences(a.n, a.length, seed)
    return seqs, ska.Dataset.synthetic(seqs, th=0.01, threads=threads)


def make_kernel(kind):
    import stem_kernel_amd as ska
    return {"ss": ska.SuStemStrKernel, "stem": ska.SuStemKernel, "stem4d": ska.StemKernel4D,
            "bpla": ska.BPLAKernel}[kind]()


# ------------------------------------------------------------------ rooflines
def dag_bytes(shapes, x, y):
    """SURVEY.md §8(d) DAG-stem model per pair:
    B = 32*|Vx|*|Vy| + S(x) + S(y) + 8,  S = 20|V| + 8|E| + 8|F| + 4L."""
    V, E, F, L = shapes[:, 0], shapes[:, 1], shapes[:, 2], shapes[:, 4]
    S = 20.0 * V + 8.0 * E + 8.0 * F + 4.0 * L
    return float(np.sum(32.0 * V[x] * V[y] + S[x] + S[y] + 8.0))


def stem4d_cells(lens, x, y):
    n, m = lens[x].astype(np.float64), lens[y].astype(np.float64)
    return float(np.sum((n + 1) * (n + 2) / 2 * (m + 1) * (m + 2) / 2))


def roofline(kind, shapes, x, y, ms):
    """(bound, achieved, unit, peak, model, algorithmic work of the launches)."""
    lens = shapes[:, 4]
    if kind in ("ss", "stem"):
        b = dag_bytes(shapes, x, y)
        return "hbm", b / (ms * 1e-3) / 1e9, "GB/s", PEAK_HBM_GBS, \
            "SURVEY §8d: 32*|Vx|*|Vy| + S(x) + S(y) + 8 bytes per pair", b
    if kind == "stem4d":
        b = 72.0 * stem4d_cells(lens, x, y)
        return "hbm", b / (ms * 1e-3) / 1e9, "GB/s", PEAK_HBM_GBS, \
            "SURVEY §8d: 72 B per (i,j,k,l) cell, [n(n+1)/2][m(m+1)/2] cells", b
    f = 24.0 * float(np.sum(lens[x].astype(np.float64) * lens[y]))
    return "valu", f / (ms * 1e-3) / 1e12, "TFLOP/s", PEAK_FP64_TFS, \
        "SURVEY §8d: 24 flop per cell (exp counted as 1), Lx*Ly cells", f


# ------------------------------------------------------------------ CPU baseline
def host_threads():
    """Host cores this process may use: its CPU affinity, capped by
    OMP_NUM_THREADS when set (the GPU box's per-job CPU share)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(cap))) if cap and cap.isdigit() else aff


def cpu_baseline(cfg, data, n_pairs, seed=7):
    """The C oracle (plain-C restatement of the reference kernels, oracle/)
    on a bounded random sample of the same Gram's pairs, host threads.
    Returns (baseline dict, sampled pairs, oracle values)."""
    from concurrent.futures import ThreadPoolExecutor

    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    rng = np.random.default_rng(seed)
    kind = cfg["kernel"]
    npool = min(len(data), 48 if kind == "stem4d" else 512)
    idx = [int(i) for i in rng.choice(len(data), size=npool, replace=False)]
    kern = make_kernel(kind)
    p = kern.params
    if kind == "stem4d":
        prep = {i: (data[i].lower(), ska.fold(data[i])) for i in idx}

        def one(ab):
            (xa, bx), (xb, by) = prep[ab[0]], prep[ab[1]]
            return po.stem4d(xa, bx, xb, by, p.gap, p.stack, p.subst, p.bp_bound, p.bp_model,
                             p.loop)
    else:
        def om_of(i):
            rows = data[i] if isinstance(data[i], list) else [data[i]]
            return po.OMData(rows, [ska.fold(r.replace("-", "")) for r in rows], 0.01)
        om = {i: om_of(i) for i in idx}

        def one(ab):
            return po.kernel_value(p.kind, om[ab[0]], om[ab[1]], p)
    pairs = []
    while len(pairs) < n_pairs:
        a, b = sorted(rng.choice(idx, size=2))
        pairs.append((int(a), int(b)))
    cores = host_threads()
    t = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:  # ctypes releases the GIL
        vals = np.array(list(ex.map(one, pairs)))
    dt = time.perf_counter() - t
    what = {"ss": "SuStemStrKernel", "stem": "SuStemKernel", "stem4d": "4-D StemKernel full_dp",
            "bpla": "BPLAKernel"}[kind]
    return {"value": n_pairs / dt, "unit": "sequence-pairs/sec", "cores": cores, "kind": "port",
            "host_nproc": os.cpu_count(),
            "sample": f"{n_pairs} random pairs (i<=j) among {npool} of the {len(data)} examples, "
                      f"{what} via the C oracle on {cores} threads (all host cores this job "
                      f"may use: affinity capped by OMP_NUM_THREADS), {dt:.1f}s wall"}, pairs, vals


# ------------------------------------------------------------------ main
def main():
    a = parse()
    cfg = CONFIGS[a.config]
    a.n = a.n or cfg["n"]
    if a.length is None:
        a.length = cfg["L"] if isinstance(cfg["L"], int) else cfg["L"][1]
    a.slices = a.slices or cfg["slices"]
    a.cpu_pairs = a.cpu_pairs or cfg["cpu_pairs"]
    kind = cfg["kernel"]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    import torch
    import torch.distributed as dist
    import stem_kernel_amd as ska

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = torch.device("cuda", local)

    # ---- inputs (identical on every rank), built on host threads
    t0 = time.perf_counter()
    data, ds = build_inputs(cfg, a)
    t_build = time.perf_counter() - t0
    stream = torch.cuda.current_stream(dev)
    ctx = ska.Context(local, stream=stream.cuda_stream)
    t0 = time.perf_counter()
    ctx.upload(ds)
    torch.cuda.synchronize(dev)
    t_upload = time.perf_counter() - t0
    shapes = np.array([ds.shape(i) for i in range(a.n)], dtype=np.float64)
    kern = make_kernel(kind)

    iu, ju = np.triu_indices(a.n)
    iu = iu.astype(np.int32)
    ju = ju.astype(np.int32)
    # the engine's own RCCL communicator (sk_comm_init; torch only carries
    # the 128-byte id from rank 0)
    from stem_kernel_amd import shard
    if dist_on:
        shard.rccl_init(ctx)
    else:
        import ctypes
        uid = ctypes.create_string_buffer(128)
        ska.lib().sk_comm_unique_id(uid, 128)
        ctx.comm_init(uid.raw, 0, 1)
    S = a.slices
    if a.full:
        a.steps, a.warmup = 1, 0
    n_slices_needed = (a.warmup + a.steps) * world
    S = max(S, n_slices_needed)
    S = -(-S // world) * world  # a multiple of N: rank r's slices are cells k % N == r
    G = S // world
    if kind in ("ss", "stem") and G <= a.n // 2:
        # folded column pairs dealt round-robin to G column groups
        colg = np.empty(a.n, np.int64)
        for p in range(a.n // 2):
            colg[p] = colg[a.n - 1 - p] = p % G
        if a.n % 2:
            colg[a.n // 2] = (a.n // 2) % G
        cell_g = colg[ju]
        kcell = np.arange(iu.size, dtype=np.int64)
        groups = {}

        def slice_of_step(t):
            g = t % G
            if g not in groups:
                groups[g] = np.flatnonzero(cell_g == g)
            sel = groups[g]
            sel = sel[kcell[sel] % world == rank]
            return iu[sel], ju[sel]
        per = max(int(np.count_nonzero(cell_g == g)) for g in range(G))
        per = -(-per // world)
        step_kind = f"column group (step mod {G}) of {G} folded-pair groups, cells k % {world} == rank"
    else:
        def slice_of_step(t):
            s = (t * world + rank) % S
            return iu[s::S], ju[s::S]
        per = int(np.ceil(iu.size / S))
        step_kind = f"cells k % {S} == step*{world} + rank"
    out = torch.zeros(per, dtype=torch.float64, device=dev)
    gathered = torch.empty(per * world, dtype=torch.float64, device=dev)
    full_gram = [None]

    def run_step(step):
        if a.full:  # the product path: sk_gram_sharded over all ranks
            full_gram[0] = ctx.gram_sharded(ds, kern, normalize=False)
            x, y = shard.rank_pairs(a.n, world, rank)
            return x, y, dict(ctx.last_timing(), **ctx.last_launch_ms())
        x, y = slice_of_step(step)
        ctx.pairs_device(ds, kern, x, y, out.data_ptr())
        tm = dict(ctx.last_timing(), **ctx.last_launch_ms())
        ctx.allgather(out.data_ptr(), per, gathered.data_ptr())
        return x, y, tm

    for w in range(a.warmup):
        run_step(w)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    local_pairs = 0
    k_ms, work, cells, launches, l_ms = [], [], [], [], []
    for k in range(a.steps):
        x, y, tm = run_step(a.warmup + k)
        local_pairs += x.size
        k_ms.append(tm["stem_ms"])
        cells.append(tm["cells"])
        launches.append(tm["launches"])
        l_ms.append(tm["ms_sum"])
        work.append((x, y))
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed, float(local_pairs)], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        total_pairs = float(sm[1])
    else:
        total_pairs = float(local_pairs)

    if rank == 0:
        value = total_pairs / elapsed
        # dominant kernel (stem / 4-D / BPLA): each launch timed by HIP events
        # around it on its own stream (sk_last_launch_ms) -- the average a
        # kernel-trace profile reports.  Launches on several streams overlap
        # (`overlap` of them on average), each then sharing the GPU, so the
        # rate is taken over the launches' span (sk_last_timing): achieved =
        # algorithmic bytes per launch / (average duration / overlap)
        tot_ms = float(np.sum(k_ms))
        sum_ms = float(np.sum(l_ms))
        xs = np.concatenate([w[0] for w in work])
        ys = np.concatenate([w[1] for w in work])
        bound, ach, unit, peak, model, alg = roofline(kind, shapes, xs, ys, tot_ms)
        n_launch = max(1, int(np.sum(launches)))
        traffic, traffic_src = None, None
        pmc_json = a.pmc_json or os.path.join(ROOT, "profiles", f"{kind}_traffic.json")
        try:
            with open(pmc_json) as f:
                pm = json.load(f)
            if pm.get("length") == a.length and pm.get("kernel") == kind:
                traffic = pm["hbm_bytes_per_cell"] * float(np.sum(cells)) / n_launch
                traffic_src = (f"not measured in this run: {os.path.relpath(pmc_json, ROOT)} "
                               f"(rocprofv3 FETCH_SIZE/WRITE_SIZE passes, {pm.get('source', '?')}) "
                               f"bytes per cell x this run's cells per launch")
        except Exception:
            pass
        cpu, parity = None, None
        if not a.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            cpu, cpairs, cvals = cpu_baseline(cfg, data, a.cpu_pairs)
            # the baseline's oracle values double as a parity check of the
            # benched kernel classes on the same inputs (1e-6 relative)
            cx = np.array([p[0] for p in cpairs], np.int32)
            cy = np.array([p[1] for p in cpairs], np.int32)
            got = ctx.pairs(ds, kern, cx, cy)
            err = float(np.max(np.abs(got - cvals) / np.maximum(np.abs(cvals), 1e-300)))
            parity = {"pairs": int(cx.size), "max_rel_err": err, "tol": 1e-6,
                      "ok": bool(err < 1e-6), "against": "C oracle (cpu_baseline sample)"}
        kname = {"ss": "sk_dag_stem_kernel", "stem": "sk_dag_stem_kernel",
                 "stem4d": "sk_stem4d_kernel", "bpla": "sk_bpla_kernel"}[kind]
        kdesc = {
            "ss": "SuStemStrKernel(alpha=0.2,beta=0.3,loop_gap=0.2,gap=0.8,band=10)",
            "stem": "SuStemKernel(beta=0.3,loop_gap=0.2,band=10)",
            "stem4d": "StemKernel<double,BPMatrix>(gap=0.8,stack=1.0,subst=0.5,bp_bound=0) full_dp",
            "bpla": "BPLAKernel(gap=-8,ext=-0.75,alpha=4.5,beta=0.11)"}[kind]
        metric = "sequence-pairs/sec (Gram entries/s) at L=200 nt" if a.config == "ns" else \
            f"sequence-pairs/sec ({a.config})"
        line = {
            "metric": metric,
            "value": value,
            "unit": "sequence-pairs/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 ACGU sequences, Nussinov-Boltzmann bpp stand-in for "
                    "ViennaRNA; no checkpoints)",
            "config": {
                "workload": f"{a.config}: {a.n}x{a.n} {kdesc} Gram, L={cfg['L']}, "
                            f"step = 1/{S} of the {iu.size} upper-triangle pairs per GPU",
                "step_cells": step_kind,
                "n_sequences": a.n, "length": cfg["L"], "pairs_per_step_per_gpu": per,
                "kernel": kdesc, "basepair_th": 0.01,
                "parallelism": f"cyclic cell plan x{world} (sk_comm_allgather, RCCL)"
                               + (" -- full Gram via sk_gram_sharded" if a.full else ""),
                "mean_nodes": float(shapes[:, 0].mean()), "mean_edges": float(shapes[:, 1].mean()),
                "mean_bpfreq": float(shapes[:, 2].mean()),
                "host_build_s": round(t_build, 2), "upload_s": round(t_upload, 3),
            },
            "roofline": {
                "bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak,
                "traffic": traffic, "traffic_source": traffic_src, "kernel": kname,
                "kernel_ms_per_launch": sum_ms / n_launch, "launches": n_launch,
                "overlap": sum_ms / tot_ms if tot_ms > 0 else None,
                "effective_ms_per_launch": tot_ms / n_launch,
                "traffic_frac": (traffic / (tot_ms / n_launch * 1e-3) / (peak * 1e9)
                                 if traffic is not None and unit == "GB/s" and tot_ms > 0 else None),
                "algorithmic_per_launch": alg / n_launch, "model": model,
                # the same bytes over the plain average launch duration (what
                # rocprof's kernel stats show), ignoring that launches overlap
                "frac_per_launch": ach / peak * tot_ms / sum_ms if sum_ms > 0 else None,
                "note": ("frac > 1: the kernel moves fewer bytes than the model counts "
                         "(rows kept in registers / LDS); measured HBM traffic is traffic_frac "
                         "of peak, so HBM no longer bounds it")
                        if ach / peak > 1.0 else None,
            },
            "cpu_baseline": cpu,
            "parity": parity,
            "cells_per_step": float(np.mean(cells)),
        }
        print(json.dumps(line), flush=True)
        if parity is not None and not parity["ok"]:
            print(f"PARITY FAILURE: max relative error {parity['max_rel_err']:.3g} > 1e-6",
                  file=sys.stderr, flush=True)
            sys.exit(3)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
