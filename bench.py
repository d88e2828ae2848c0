#!/usr/bin/env python3
"""Benchmark: stem-kernel Gram matrix (north star) on MI355X.

Workload (BASELINE.json north_star / metric): the 4096 x 4096 Gram matrix of
SuStemStrKernel (== StemStrKernel of stem_kernel_lite/ss_kernel.h: DAG stem
kernel + profile string kernel, default parameters of
stem_kernel_lite/main.cpp:103-149) over synthetic RNA sequences of L = 200 nt
(splitmix64 sequences, Nussinov-Boltzmann base-pairing probabilities,
--basepair 0.01).  Units are Gram cells K(i,j), i <= j, exactly the cells the
reference evaluates (common/kernel_matrix.cpp:44-55): 8,390,656 sequence pairs.

A *step* is one slice of that upper triangle: the pairs are dealt round-robin
into S = --slices equal slices (default 64, ~131k pairs each), so every
slice has the same cost mix.  With N GPUs (one process per GPU, RCCL), rank r
computes slice (step*N + r) -- per-GPU work is fixed, so scaling is weak -- and
the ranks all-gather the step's Gram entries over RCCL (the reference
gathered to rank 0 with MPI point-to-point, kernel_matrix.cpp:225-261).
--full runs every slice of the Gram once (whole job).

Timed region: inputs (packed DAGs) already resident in HBM; each step = the
DAG stem DP + string DP + combine epilogue for the slice + the all-gather.
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

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
CONFIG_ID = 2           # seed 0x5EED0000 + config id (north star shares C3's L)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=4096, help="number of sequences")
    ap.add_argument("--length", type=int, default=200)
    ap.add_argument("--slices", type=int, default=64)
    ap.add_argument("--full", action="store_true", help="time every slice (whole Gram)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-pairs", type=int, default=12288, help="pairs in the CPU sample (~15 s on 16 cores)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "stem_traffic.json"))
    return ap.parse_args()


def algorithmic_bytes(shapes, x, y):
    """SURVEY.md §8(d) DAG-stem model per pair:
    B = 32*|Vx|*|Vy| + S(x) + S(y) + 8,  S = 20|V| + 8|E| + 8|F| + 4L."""
    V, E, F, L = shapes[:, 0], shapes[:, 1], shapes[:, 2], shapes[:, 4]
    S = 20.0 * V + 8.0 * E + 8.0 * F + 4.0 * L
    return float(np.sum(32.0 * V[x] * V[y] + S[x] + S[y] + 8.0))


def cpu_baseline(seqs, n_pairs, seed=7):
    """The C oracle (plain-C restatement of the reference kernels, oracle/)
    on a bounded random sample of the same Gram's pairs, host threads."""
    from concurrent.futures import ThreadPoolExecutor

    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    rng = np.random.default_rng(seed)
    idx = rng.choice(len(seqs), size=min(len(seqs), 48), replace=False)
    om = {int(i): po.OMData([seqs[i]], [ska.fold(seqs[i])], 0.01) for i in idx}
    pairs = []
    while len(pairs) < n_pairs:
        a, b = sorted(rng.choice(idx, size=2))
        pairs.append((int(a), int(b)))
    p = ska.SuStemStrKernel().params
    cores = max(1, min(16, os.cpu_count() or 1))

    def one(ab):
        return po.kernel_value(p.kind, om[ab[0]], om[ab[1]], p)

    t = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:  # ctypes releases the GIL
        list(ex.map(one, pairs))
    dt = time.perf_counter() - t
    return {"value": n_pairs / dt, "unit": "sequence-pairs/sec", "cores": cores, "kind": "port",
            "sample": f"{n_pairs} random pairs (i<=j) among 48 of the {len(seqs)} L={len(seqs[0])} "
                      f"sequences, SuStemStrKernel via the C oracle, {dt:.1f}s wall"}


def main():
    a = parse()
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
    seqs = ska.random_sequences(a.n, a.length, 0x5EED0000 + CONFIG_ID)
    ds = ska.Dataset.synthetic(seqs, th=0.01, threads=min(16, os.cpu_count() or 1))
    t_build = time.perf_counter() - t0
    stream = torch.cuda.current_stream(dev)
    ctx = ska.Context(local, stream=stream.cuda_stream)
    t0 = time.perf_counter()
    ctx.upload(ds)
    torch.cuda.synchronize(dev)
    t_upload = time.perf_counter() - t0
    shapes = np.array([ds.shape(i) for i in range(a.n)], dtype=np.float64)
    kern = ska.SuStemStrKernel()

    iu, ju = np.triu_indices(a.n)
    iu = iu.astype(np.int32)
    ju = ju.astype(np.int32)
    S = a.slices
    n_slices_needed = (a.warmup + a.steps) * world
    if a.full:
        S = max(world, S)
        a.steps = S // world
        a.warmup = 0
        n_slices_needed = S
    if n_slices_needed > S:
        S = n_slices_needed
    slice_of = lambda s: (iu[s::S], ju[s::S])
    per = int(np.ceil(iu.size / S))
    out = torch.empty(per, dtype=torch.float64, device=dev)
    gathered = torch.empty(per * world, dtype=torch.float64, device=dev)

    stem_ms = []
    cells = []
    alg_bytes = []
    pairs_done = 0

    def run_step(step):
        nonlocal pairs_done
        sl = step * world + rank
        x, y = slice_of(sl % S)
        ctx.pairs_device(ds, kern, x, y, out.data_ptr())
        tm = ctx.last_timing()
        if dist_on:
            dist.all_gather_into_tensor(gathered, out)
        return x.size, tm

    for w in range(a.warmup):
        run_step(w)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    local_pairs = 0
    for k in range(a.steps):
        n_p, tm = run_step(a.warmup + k)
        local_pairs += n_p
        stem_ms.append(tm["stem_ms"])
        x, y = slice_of(((a.warmup + k) * world + rank) % S)
        alg_bytes.append(algorithmic_bytes(shapes, x, y))
        cells.append(tm["cells"])
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
        # dominant kernel: DAG stem DP, per launch (one launch per step)
        st_ms = float(np.mean(stem_ms))
        ach = float(np.mean(alg_bytes)) / (st_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(a.pmc_json) as f:
                pm = json.load(f)
            if pm.get("length") == a.length:
                traffic = pm["hbm_bytes_per_cell"] * float(np.mean(cells))
        except Exception:
            pass
        cpu = None
        if not a.no_cpu_baseline:
            cpu = cpu_baseline(seqs, a.cpu_pairs)
        line = {
            "metric": "sequence-pairs/sec (Gram entries/s) at L=200 nt",
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
                "workload": f"{a.n}x{a.n} SuStemStrKernel (ss_kernel) Gram, L={a.length}, "
                            f"step = 1/{S} of the {iu.size} upper-triangle pairs per GPU",
                "n_sequences": a.n, "length": a.length, "pairs_per_step_per_gpu": per,
                "kernel": "SuStemStrKernel(alpha=0.2,beta=0.3,loop_gap=0.2,gap=0.8,band=10)",
                "basepair_th": 0.01, "parallelism": f"gram-slices x{world} (RCCL all-gather)",
                "mean_nodes": float(shapes[:, 0].mean()), "mean_edges": float(shapes[:, 1].mean()),
                "mean_bpfreq": float(shapes[:, 2].mean()),
                "host_build_s": round(t_build, 2), "upload_s": round(t_upload, 3),
            },
            "roofline": {
                "bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": ach / PEAK_HBM_GBS,
                "traffic": traffic,
                "kernel": "sk_dag_stem_kernel", "kernel_ms_per_launch": st_ms,
                "model": "SURVEY §8d: 32*|Vx|*|Vy| + S(x) + S(y) + 8 bytes per pair",
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
