#!/usr/bin/env python3
"""Benchmark of the stem-kernel Gram engine on MI355X.

Default workload (BASELINE.json north_star / metric, ``--config ns``): the
4096 x 4096 Gram matrix of LSuStemStrKernel -- the reference CLI's --log mode
(stem_kernel_lite/main.cpp:187-191; its plain SuStemStrKernel default never
runs, :180-186): beta*log(DAG stem kernel) + alpha*log(profile string kernel),
default parameters of stem_kernel_lite/main.cpp:103-149 -- over synthetic RNA
sequences of L = 200 nt (splitmix64 sequences, Nussinov-Boltzmann
base-pairing probabilities, --basepair 0.01).  Units are Gram cells K(i,j),
i <= j, exactly the cells the reference evaluates
(common/kernel_matrix.cpp:44-55): 8,390,656 sequence pairs.

A *step* is one slice of that upper triangle, 1/S of its cells per GPU.  The
product's sharded Gram (sk_gram_sharded, the reference MPI Gram's cyclic plan,
kernel_matrix.cpp:210-224) gives rank r of N the cells k % N == r (k =
row-major index of cell (i, j), i <= j), and every slice is a subset of that
plan, so over S/N steps a rank computes exactly its share of the shipped
Gram.  DAG and BPLA kernels (ns, c2, c5, c4): the columns j (the y examples) are folded in
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

Ranks: under torchrun (RANK set) each process is one rank; ``--gpus N``
without a launcher starts its own N worker processes (spawn_ranks) before any
GPU call, so ``python3 bench.py --gpus 8`` runs as-is.

Roofline: see roofline() -- measured HBM bytes (profiles/<config>_traffic.json,
stamped with the kernel source hash; stale profiles are not used) over the
launches' span for the HBM-bound kernels, the survey model beside it
(profiles/<config>_traffic.json, stamped with the kernel source hash).
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

# name -> kernel family, n examples, length, slices, config id (seed
# 0x5EED0000+id); `cls` overrides the family's kernel class.  NS runs the
# reference CLI's --log mode (LSuStemStrKernel, stem_kernel_lite/main.cpp:
# 187-191): plain SuStemStrKernel is the CLI's dead default (it prints a memory
# estimate and returns, :180-186), and in the --log composition both DPs reach
# the written Gram (in the plain sum the stem term is ~1e-32 of the string
# term at L=200).  Same two DPs, plus a log epilogue in sk_combine_kernel.
CONFIGS = {
    # NS: a step is 1/8 of the Gram (1.05M pairs, 4.8 s): 219.9k / 219.8k
    # pairs/s against 218.4k / 218.3k with 1/16 on one box (r06u; r05w: 1/16
    # 206.2k, 1/24 203.7k, 1/48 201.2k -- the class launches' fill and last
    # round over more pairs); the whole Gram in one call (sk_gram_sharded,
    # bench --full) 220.0k (r06s); 8 divides the driver's 1, 2, 4 and 8 GPUs
    # (asynchronous calls, below: +0.7 %, r06q)
    "ns": dict(kernel="ss", cls="LSuStemStrKernel", n=4096, L=200, slices=8, cid=2, cpu_pairs=12288,
               async_calls=True),
    # C2's whole Gram is 32,896 pairs (0.2 s): a step is the whole Gram, the
    # unit the reference computes per call (kernel_matrix.cpp:485-575), not a
    # slice whose launch fill and tail would dominate ("whole": steps repeat it)
    # (asynchronous: 261.3k / 262.1k against 259.4k / 259.6k, r06ab; C3 gains
    # nothing from it, 1,590-1,591 either way, and stays synchronous)
    "c2": dict(kernel="ss", n=256, L=150, slices=1, whole=True, cid=1, cpu_pairs=12288, async_calls=True),
    # C3: 1,023 pairs per step, one workgroup per pair (LDS: one per CU), so
    # four rounds of 256 CUs: 591.8 / 755.2 / 759.5 pairs/s for 384 / 768 /
    # 1,023 pairs on one box (r05j, an earlier column kernel; 384 leaves half
    # the CUs idle in its second round)
    "c3": dict(kernel="stem4d", n=1024, L=200, slices=513, cid=2, cpu_pairs=32),
    # async: step t+1 planned while step t runs (sk_set_async): C4 +3.6 % (its
    # 7 ms steps had 0.6-0.9 ms host gaps); NS +0.7 % (214.9k / 214.9k against
    # 213.2k / 213.4k) and C5 +0.4 % (r06q: the ≈ 25 ms gap between steps --
    # the all-gather, then the next step's host planning -- is hidden); the
    # roofline's time base is the launches' span either way
    # C4: a step is 1/6 of the Gram (350k pairs): 20.5-20.8M against 18.5M
    # pairs/s with 1/16 steps on one box (r04u / r04v: the launch's fill and
    # last round of items amortized over 2.7x the work)
    "c4": dict(kernel="bpla", n=2048, L=(190, 210), rows=4, slices=6, cid=3, cpu_pairs=196608, async_calls=True),
    # C5: 1/64 of the Gram per step (525k pairs; 110.2k against 109.0k pairs/s
    # with 1/128 on one box, r04w2)
    "c5": dict(kernel="stem", n=8192, L=300, slices=64, cid=4, cpu_pairs=4096, async_calls=True),
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
    ap.add_argument("--sync", action="store_true", help="synchronous compute calls for every config")
    ap.add_argument("--async", dest="async_calls", action="store_true",
                    help="asynchronous compute calls (sk_set_async) for every config (default: C4 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-pairs", type=int, default=None, help="pairs in the CPU sample")
    ap.add_argument("--pmc-json", default=None, help="traffic profile (default profiles/<kind>_traffic.json)")
    ap.add_argument("--cpu-stub", default=None, metavar="MODULE:FUNC",
                    help="test harness: FUNC(data, params, x, y) compute + gloo all-gather instead of "
                         "the GPU (no measurement)")
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


def make_kernel(kind, cls=None):
    import stem_kernel_amd as ska
    if cls:
        return getattr(ska, cls)()
    return {"ss": ska.SuStemStrKernel, "stem": ska.SuStemKernel, "stem4d": ska.StemKernel4D,
            "bpla": ska.BPLAKernel}[kind]()


def components(kern):
    """The component kernels of a stem + string composition (def_kernel.h:
    86-111, 165-190): the DAG stem DP (SuStemKernel) and the profile string
    kernel (StringKernel) with the composition's own parameters, so each DP is
    checked on its own -- in a plain sum the stem term is invisible."""
    import stem_kernel_amd as ska
    from stem_kernel_amd import _lib
    p = kern.params
    if p.kind in (_lib.SU_STEM_STR, _lib.LSU_STEM_STR):
        return {"stem": ska.SuStemKernel(loop_gap=p.loop_gap, beta=p.beta, len_band=p.len_band),
                "string": ska.StringKernel(gap=p.gap, alpha=p.alpha)}
    return {}


def compose(kind, p, stem, string):
    """def_kernel.h:86-111 (SuStemStr: K_stem + K_str) and :165-190
    (LSuStemStr: beta*log K_stem + alpha*log K_str), from the components,
    in oracle/pyoracle.py kernel_value's operation order."""
    import math

    from stem_kernel_amd import _lib
    if kind == _lib.SU_STEM_STR:
        return stem + string
    if kind == _lib.LSU_STEM_STR:
        return (p.beta * math.log(stem) + 0.0) + (p.alpha * math.log(string) + 0.0)
    raise ValueError(kind)


# ------------------------------------------------------------------ rooflines
def dag_bytes(shapes, x, y):
    """SURVEY.md §8(d) DAG-stem model per pair:
    B = 32*|Vx|*|Vy| + S(x) + S(y) + 8,  S = 20|V| + 8|E| + 8|F| + 4L."""
    V, E, F, L = shapes[:, 0], shapes[:, 1], shapes[:, 2], shapes[:, 4]
    S = 20.0 * V + 8.0 * E + 8.0 * F + 4.0 * L
    return float(np.sum(32.0 * V[x] * V[y] + S[x] + S[y] + 8.0))


def col_shape(lens, y):
    """(NB, W) of the 4-D column kernel as run_stem4d picks them for a batch
    (sk_stem4d_col_shape: NB chained columns per group by class, W waves per
    pair bounded by m - 2 PF - 2 of the smallest y, registers and LDS; one
    batch per bench step)."""
    from stem_kernel_amd.kernel_matrix import stem4d_col_shape
    m = lens[y]
    big = m[m >= 2]
    sh = stem4d_col_shape(int(big.min()) if big.size else 0, int(m.max()))
    return sh["nb"], sh["waves"]


def stem4d_cells(lens, x, y):
    n, m = lens[x].astype(np.float64), lens[y].astype(np.float64)
    return float(np.sum((n + 1) * (n + 2) / 2 * (m + 1) * (m + 2) / 2))


def dag_row_bytes(rt, x, y):
    """Row transfers of the DAG stem kernel's gamma schedule,
    from sk_dataset_row_traffic: per pair (x, y) every transfer of one of x's
    rows moves 8 * y_slots(y) bytes.  (lower, schedule): the compulsory bytes
    -- each stored row written once and read back once (a second parent's
    read could be an L2 hit) -- and every transfer the schedule issues
    (stored rows, slab / Gamma / Phi child-row reads; register-held rows
    move nothing)."""
    slot_b = 8.0 * rt[y, 6]
    lower = float(np.sum(slot_b * 2.0 * rt[x, 1]))
    sched = float(np.sum(slot_b * (rt[x, 1] + rt[x, 2] + rt[x, 3] + rt[x, 4])))
    return lower, sched


def algorithmic(kind, shapes, x, y, rt=None):
    """(bound, unit, peak, model description, algorithmic work of the pairs,
    extra model figures)."""
    lens = shapes[:, 4]
    if kind in ("ss", "stem"):
        survey = dag_bytes(shapes, x, y)
        if rt is None:
            return "hbm", "GB/s", PEAK_HBM_GBS, \
                "SURVEY §8d: 32*|Vx|*|Vy| + S(x) + S(y) + 8 bytes per pair", survey, {}
        lower, sched = dag_row_bytes(rt, x, y)
        return "hbm", "GB/s", PEAK_HBM_GBS, \
            "compulsory row traffic of the gamma schedule: 2 x 8 B x y_slots(y) per row of x stored " \
            "in the HBM slab (written once, read back once; sk_dataset_row_traffic, DESIGN.md §6)", lower, \
            {"schedule_bytes": sched, "survey_model_bytes": survey}
    if kind == "stem4d":
        if os.environ.get("SK4_NO_GSUM"):  # the four-state planes (A/B switch)
            return "hbm", "GB/s", PEAK_HBM_GBS, \
                "SURVEY §8d: 72 B per (i,j,k,l) cell, [n(n+1)/2][m(m+1)/2] cells", \
                72.0 * stem4d_cells(lens, x, y), {}
        col = not (os.environ.get("SK4_SPAN") or os.environ.get("SK4_NO_PRE"))
        if col and int(lens[y].max()) + 1 <= 512:
            # column groups (stem4d.hip sk_stem4d_col_kernel): G0 of (i, j_lo-1)
            # read by a group's first chain and G0 of (i, j_hi) written by its
            # last (16 B per NB columns); every W-th position's pre-combined G1
            # crosses the round wrap through HBM (16 B)
            NB, W = col_shape(lens, y)
            return "hbm", "GB/s", PEAK_HBM_GBS, \
                f"16/NB B per (i,j,k,l) cell (G0 read by a group's first column, written by its last; " \
                f"NB = {NB}) + 16/W B (W = {W}: every W-th position's pre-combined G1 across the round " \
                "wrap), [n(n+1)/2][m(m+1)/2] cells", (16.0 / NB + 16.0 / W) * stem4d_cells(lens, x, y), {}
        if os.environ.get("SK4_NO_PRE") or int(lens[y].max()) + 1 > 512:
            # full_dp with the K chain summed (stem4d.hip): G0, G1 written once
            # (16 B), G0 of (i,j-1), G1 of (i+1,j) and the stacking G0 of
            # (i+1,j-1) read once (24 B); SURVEY §8d's 72 B counted K0, K1 too
            # (|y| > 511: k tiles, which keep this kernel)
            return "hbm", "GB/s", PEAK_HBM_GBS, \
                "40 B per (i,j,k,l) cell (G0, G1 written; G0, G1, stacking G0 read; SURVEY §8d's 72 B " \
                "less the K states, which are summed), [n(n+1)/2][m(m+1)/2] cells", \
                40.0 * stem4d_cells(lens, x, y), {}
        # + each plane's stacking chain produced one span early (pre-combined G1)
        return "hbm", "GB/s", PEAK_HBM_GBS, \
            "32 B per (i,j,k,l) cell (G0 and the consumer's pre-combined G1 written, G0 and the own " \
            "pre-combined G1 read; SURVEY §8d's 72 B less the summed K states and the stacking read), " \
            "[n(n+1)/2][m(m+1)/2] cells", 32.0 * stem4d_cells(lens, x, y), {}
    return "valu", "TFLOP/s", PEAK_FP64_TFS, \
        "SURVEY §8d: 24 flop per cell (exp counted as 1), Lx*Ly cells", \
        24.0 * float(np.sum(lens[x].astype(np.float64) * lens[y])), {}


def load_profile(config, kind, length, path=None):
    """profiles/<config>_traffic.json (tools/measure.sh -> tools/profile_summary.py)
    and whether it was measured on these kernel sources (provenance hash)."""
    from stem_kernel_amd import provenance
    path = path or os.path.join(ROOT, "profiles", f"{config}_traffic.json")
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None, None, path
    if pm.get("kernel") != kind or pm.get("length") != length:
        return None, None, path
    return pm, pm.get("source_hash") == provenance.source_hash(), path


def roofline(config, kind, length, shapes, xs, ys, span_ms, sum_ms, n_launch, cells, pmc_json=None, rt=None):
    """The dominant kernel's roofline.

    HBM-bound kernels (DAG stem, 4-D stem): the headline `achieved` is the
    implemented algorithm's COMPULSORY bytes per launch
    (`algorithmic_per_launch`: DAG, the gamma schedule's stored rows written
    and read back once, `dag_row_bytes`; 4-D column kernel, 16/NB + 16/W B per
    cell) over the launches' span per launch (the launches run on several
    streams and overlap: span / launches), so `frac` is the compulsory-traffic
    fraction of the 8 TB/s peak.  The counter figure stands beside it:
    `traffic` (rocprofv3 2 x FETCH_SIZE + WRITE_SIZE per launch, per cell from
    the committed profile, scaled to this run's cells) and `traffic_frac`
    (traffic over the same span) -- L2-to-fabric bytes, Infinity-Cache (MALL)
    hits included (MI355X_MICROARCH.md; tools/calib/fetch_calib.hip's
    re-read case), so an upper bound of the HBM bytes, not HBM bytes.  The
    DAG kernel also reports every row transfer its schedule issues
    (`schedule_bytes_per_launch`) and SURVEY §8d's model bytes
    (`survey_model_bytes_per_launch`, no fraction: the path-sum, gamma and phi
    reformulation never moves them).  A profile measured on other kernel
    sources is `stale`: its `traffic` is then null.  `frac_per_avg_launch`
    puts the compulsory bytes over the average launch duration instead of the
    span.  FP64 kernels (BPLA): algorithmic flops per launch over the average
    launch duration."""
    bound, unit, peak, model, alg, extra = algorithmic(kind, shapes, xs, ys, rt)
    n_launch = max(1, n_launch)
    avg_s = sum_ms / n_launch * 1e-3
    eff_s = span_ms / n_launch * 1e-3
    alg_pl = alg / n_launch
    scale = 1e9 if unit == "GB/s" else 1e12
    pm, fresh, path = load_profile(config, kind, length, pmc_json)
    rel = os.path.relpath(path, ROOT)
    traffic = None
    if pm is not None and pm.get("hbm_bytes_per_cell"):
        traffic = pm["hbm_bytes_per_cell"] * float(np.sum(cells)) / n_launch
    r = {"bound": bound, "peak": peak, "unit": unit, "kernel": None,
         "kernel_ms_per_launch": avg_s * 1e3, "launches": n_launch,
         "overlap": sum_ms / span_ms if span_ms > 0 else None,
         "effective_ms_per_launch": eff_s * 1e3,
         "algorithmic_per_launch": alg_pl, "model": model,
         "profile": rel if pm is not None else None,
         "profile_source_hash": pm.get("source_hash") if pm else None,
         "profile_git_head": pm.get("git_head") if pm else None,
         "stale": (not fresh) if pm is not None else None}
    for k, v in extra.items():
        r[k + "_per_launch"] = v / n_launch
    if bound == "hbm":
        r["achieved"] = alg_pl / eff_s / scale if eff_s > 0 else 0.0
        r["basis"] = "compulsory (algorithmic) bytes per launch / (launches' span / launches)"
        r["frac_per_avg_launch"] = alg_pl / avg_s / scale / peak if avg_s > 0 else None
        if traffic is not None and fresh and eff_s > 0:
            r["traffic"] = traffic
            r["traffic_frac"] = traffic / eff_s / scale / peak
            r["traffic_basis"] = ("2 x FETCH_SIZE + WRITE_SIZE per launch (" + rel + ") / (launches' span / "
                                  "launches): L2-to-fabric bytes, Infinity-Cache (MALL) hits included -- an "
                                  "upper bound of the HBM bytes")
        else:
            r["traffic"] = None
            r["traffic_frac"] = None
            if traffic is not None:
                r["traffic_stale_value"] = traffic
        r["traffic_per_cell"] = pm.get("hbm_bytes_per_cell") if pm else None
        r["algorithmic_per_cell"] = alg / float(np.sum(cells)) if np.sum(cells) else None
    else:
        r["achieved"] = alg_pl / avg_s / scale if avg_s > 0 else 0.0
        r["basis"] = "algorithmic flops per launch / average launch duration"
        r["traffic"] = traffic if fresh else None
    r["frac"] = r["achieved"] / peak
    lds = (pm or {}).get("lds")
    if lds:
        r["issue"] = {"fresh": bool(fresh), "lds_busy_frac": lds.get("lds_busy_frac"),
                      "lds_bank_conflict_share": lds.get("bank_conflict_share"),
                      "valu_per_cell": lds.get("valu_per_cell"),
                      "salu_per_cell": lds.get("salu_per_cell"),
                      "lds_insts_per_cell": lds.get("lds_insts_per_cell"),
                      "source": rel + " (rocprofv3 --pmc SQ_LDS_IDX_ACTIVE ... GRBM_GUI_ACTIVE pass)"}
    return r


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
    Returns (baseline dict, sampled pairs, oracle values, oracle values of
    each component DP of a composition)."""
    from concurrent.futures import ThreadPoolExecutor

    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    rng = np.random.default_rng(seed)
    kind = cfg["kernel"]
    npool = min(len(data), 48 if kind == "stem4d" else 512)
    idx = [int(i) for i in rng.choice(len(data), size=npool, replace=False)]
    kern = make_kernel(kind, cfg.get("cls"))
    p = kern.params
    split = bool(components(kern))
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

        if split:  # the two DPs of the composition, each kept for parity
            def one(ab):
                x, y = om[ab[0]], om[ab[1]]
                return (po.kernel_value(0, x, y, p), po.kernel_value(2, x, y, p))
        else:
            def one(ab):
                return po.kernel_value(p.kind, om[ab[0]], om[ab[1]], p)
    pairs = []
    while len(pairs) < n_pairs:
        a, b = sorted(rng.choice(idx, size=2))
        pairs.append((int(a), int(b)))
    cores = host_threads()
    t = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:  # ctypes releases the GIL
        vals = list(ex.map(one, pairs))
        if split:
            comp = {"stem": np.array([v[0] for v in vals]), "string": np.array([v[1] for v in vals])}
            vals = np.array([compose(p.kind, p, a, b) for a, b in vals])
        else:
            comp, vals = {}, np.array(vals)
    dt = time.perf_counter() - t
    what = cfg.get("cls") or {"ss": "SuStemStrKernel", "stem": "SuStemKernel",
                              "stem4d": "4-D StemKernel full_dp", "bpla": "BPLAKernel"}[kind]
    value = n_pairs / dt
    return {"value": value, "unit": "sequence-pairs/sec", "cores": cores, "kind": "port",
            "host_nproc": os.cpu_count(),
            "cores_why": ("the job's CPU share: the GPU box caps each job at OMP_NUM_THREADS (16) of its "
                          f"{os.cpu_count()} host threads, which other jobs share"),
            "calibration": calibration(cfg, value, cores),
            "sample": f"{n_pairs} random pairs (i<=j) among {npool} of the {len(data)} examples, "
                      f"{what} via the C oracle on {cores} threads (all host cores this job "
                      f"may use: affinity capped by OMP_NUM_THREADS), {dt:.1f}s wall"}, pairs, vals, comp


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def calibration(cfg, value, cores):
    """How the port relates to the reference's own CPU code
    (profiles/r04_cpu_calibration.json, tools/cpu_calib.py): on one core of
    the build container the port runs the L=200 DAG stem DP `port_over_reference`
    times as fast as the reference's stem_kernel_lite/stem_kernel.cpp did in
    the survey's probe (BASELINE.md, 57 ms per pair).  The GPU box's CPU is
    another model, so only the port's rate is measured here; the reference's
    rate on these cores is estimated as value / port_over_reference."""
    path = os.path.join(ROOT, "profiles", "r04_cpu_calibration.json")
    try:
        with open(path) as f:
            c = json.load(f)
    except (OSError, ValueError):
        return None
    out = {"source": os.path.relpath(path, ROOT), "box_cpu_model": cpu_model(),
           "container_cpu_model": c.get("cpu_model"),
           "port_over_reference_in_container": c.get("port_over_reference"),
           "port_pairs_per_s_per_thread_here": value / max(cores, 1)}
    if cfg["kernel"] in ("ss", "stem") and cfg["L"] == 200 and c.get("port_over_reference"):
        out["reference_equivalent_value"] = value / c["port_over_reference"]
        out["box_over_container_per_core"] = (value / max(cores, 1)) / c["port_pairs_per_s_per_core"]
        out["note"] = ("reference_equivalent_value assumes the port/reference ratio measured in the "
                       "container holds on the box's CPU model, which is unverified")
    return out


# ------------------------------------------------------------------ ranks
def spawn_ranks(a):
    """`--gpus N` started without a launcher (RANK unset): start N fresh
    worker processes of this script -- before this process makes any GPU call
    -- with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT set, one GPU each, and exit with the first failing rank's
    status (the others are then stopped: a rank that died leaves its peers
    waiting in a collective).  The reference's MPI Gram is launched by mpirun
    the same way (common/kernel_matrix.cpp:495-527)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, start_new_session=True))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in live:
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
    return rc


class GpuEngine:
    """The product path: one GPU per rank, the engine's C ABI, its own RCCL
    communicator (sk_comm_init; torch.distributed only carries the 128-byte id
    from rank 0)."""

    def __init__(self, a, cfg, rank, world, local):
        import torch
        import torch.distributed as dist

        import stem_kernel_amd as ska
        from stem_kernel_amd import shard
        self.torch, self.dist, self.ska, self.a = torch, dist, ska, a
        self.dist_on = world > 1
        if self.dist_on:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", rank=rank, world_size=world)
        self.dev = torch.device("cuda", local)
        t0 = time.perf_counter()
        self.data, self.ds = build_inputs(cfg, a)
        self.t_build = time.perf_counter() - t0
        stream = torch.cuda.current_stream(self.dev)
        self.ctx = ska.Context(local, stream=stream.cuda_stream)
        t0 = time.perf_counter()
        self.ctx.upload(self.ds)
        torch.cuda.synchronize(self.dev)
        self.t_upload = time.perf_counter() - t0
        self.kern = make_kernel(cfg["kernel"], cfg.get("cls"))
        # asynchronous calls: the host plans step t+1 while the GPU runs step
        # t; timings are collected over the timed steps (totals())
        self.async_on = not a.sync and bool(a.async_calls or cfg.get("async_calls"))
        self.ctx.set_async(self.async_on)
        if self.dist_on:
            shard.rccl_init(self.ctx)
        else:
            import ctypes
            uid = ctypes.create_string_buffer(128)
            ska.lib().sk_comm_unique_id(uid, 128)
            self.ctx.comm_init(uid.raw, 0, 1)
        self.world, self.rank = world, rank

    def alloc(self, per):
        t = self.torch
        self.per = per
        self.out = t.zeros(per, dtype=t.float64, device=self.dev)
        self.gathered = t.empty(per * self.world, dtype=t.float64, device=self.dev)

    def step(self, x, y):
        self.ctx.pairs_device(self.ds, self.kern, x, y, self.out.data_ptr())
        tm = None if self.async_on else dict(self.ctx.last_timing(), **self.ctx.last_launch_ms())
        self.ctx.allgather(self.out.data_ptr(), self.per, self.gathered.data_ptr())
        return tm

    def full(self):
        self.ctx.gram_sharded(self.ds, self.kern, normalize=False)
        return None if self.async_on else dict(self.ctx.last_timing(), **self.ctx.last_launch_ms())

    def totals(self):
        """Summed timings of the calls since the last totals() (async mode;
        after a sync)."""
        self.ctx.sync_timing()
        return dict(self.ctx.last_timing(), **self.ctx.last_launch_ms())

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def barrier(self):
        if self.dist_on:
            self.dist.barrier()

    def reduce_max_sum(self, elapsed, pairs):
        t = self.torch.tensor([elapsed, float(pairs)], dtype=self.torch.float64, device=self.dev)
        mx, sm = t.clone(), t.clone()
        self.dist.all_reduce(mx, op=self.dist.ReduceOp.MAX)
        self.dist.all_reduce(sm, op=self.dist.ReduceOp.SUM)
        return float(mx[0]), float(sm[1])

    def close(self):
        if self.dist_on:
            self.dist.destroy_process_group()


class CpuStubEngine(GpuEngine):
    """--cpu-stub MODULE:FUNC -- the same ranks, plan, timing and JSON line
    with the GPU compute replaced by FUNC(data, kernel_params, x, y) -> values
    (a test supplies it, e.g. tests/bench_stub.py over the C oracle) and the
    all-gather by torch.distributed over gloo: exercises the N-rank bench path
    on a machine without a GPU.  After the timed steps the last step's
    gathered buffers are checked slice by slice against FUNC on every rank's
    cells.  Not a measurement (no roofline, no CPU baseline)."""

    def __init__(self, a, cfg, rank, world, local):
        import importlib

        import torch
        import torch.distributed as dist

        import stem_kernel_amd as ska
        mod, fn = a.cpu_stub.split(":")
        self.compute = getattr(importlib.import_module(mod), fn)
        self.torch, self.dist, self.ska, self.a = torch, dist, ska, a
        self.dist_on = world > 1
        if self.dist_on:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        t0 = time.perf_counter()
        self.data, self.ds = build_inputs(cfg, a)
        self.t_build = time.perf_counter() - t0
        self.t_upload = 0.0
        self.kern = make_kernel(cfg["kernel"], cfg.get("cls"))
        self.world, self.rank = world, rank
        self.checked = 0

    def values(self, x, y):
        return np.asarray(self.compute(self.data, self.kern.params, x, y), dtype=np.float64)

    def alloc(self, per):
        self.per = per

    def step(self, x, y):
        t = self.torch
        buf = t.zeros(self.per, dtype=t.float64)
        buf[: x.size] = t.from_numpy(self.values(x, y))
        parts = [t.empty(self.per, dtype=t.float64) for _ in range(self.world)]
        if self.dist_on:
            self.dist.all_gather(parts, buf)
        else:
            parts[0].copy_(buf)
        self.last = parts
        return {"stem_ms": 1e-3, "ms_sum": 1e-3, "launches": 1, "cells": float(x.size)}

    def verify(self, slice_of_rank):
        """Every rank's gathered slice of the last step equals FUNC on it."""
        for r in range(self.world):
            rx, ry = slice_of_rank(r)
            if not np.array_equal(self.last[r][: rx.size].numpy(), self.values(rx, ry)):
                raise AssertionError(f"cpu stub: rank {r}'s gathered slice differs")
            self.checked += rx.size

    def full(self):
        raise SystemExit("--full is the GPU product path (sk_gram_sharded)")

    def sync(self):
        pass

    def reduce_max_sum(self, elapsed, pairs):
        t = self.torch.tensor([elapsed, float(pairs)], dtype=self.torch.float64)
        mx, sm = t.clone(), t.clone()
        self.dist.all_reduce(mx, op=self.dist.ReduceOp.MAX)
        self.dist.all_reduce(sm, op=self.dist.ReduceOp.SUM)
        return float(mx[0]), float(sm[1])


# ------------------------------------------------------------------ plan
def make_plan(kind, n, world, rank, S):
    """Step slices of the shipped cyclic plan (cells k % world == rank).
    Returns (slice_of(step, rank) -> (x, y), per: buffer size, description)."""
    iu, ju = np.triu_indices(n)
    iu = iu.astype(np.int32)
    ju = ju.astype(np.int32)
    G = S // world
    kcell = np.arange(iu.size, dtype=np.int64)
    if kind in ("ss", "stem", "bpla") and G <= n // 2:
        # folded column pairs (j, n-1-j) dealt round-robin to G column groups
        colg = np.empty(n, np.int64)
        for p in range(n // 2):
            colg[p] = colg[n - 1 - p] = p % G
        if n % 2:
            colg[n // 2] = (n // 2) % G
        cell_g = colg[ju]
        # every group's cells at once (a stable sort by group keeps cell order)
        order = np.argsort(cell_g, kind="stable")
        bounds = np.searchsorted(cell_g[order], np.arange(G + 1))
        groups = [order[bounds[g]:bounds[g + 1]] for g in range(G)]
        cache = {}

        def slice_of(t, r=rank):
            key = (t % G, r)
            if key not in cache:
                sel = groups[t % G]
                if world > 1:
                    sel = sel[kcell[sel] % world == r]
                cache[key] = (np.ascontiguousarray(iu[sel]), np.ascontiguousarray(ju[sel]))
            return cache[key]
        # exact buffer size: the largest (group, rank) share
        per = int(np.bincount(cell_g * world + kcell % world, minlength=G * world).max())
        desc = f"column group (step mod {G}) of {G} folded-pair groups, cells k % {world} == rank"
    else:
        cache = {}

        def slice_of(t, r=rank):
            s = (t * world + r) % S
            if s not in cache:
                cache[s] = (np.ascontiguousarray(iu[s::S]), np.ascontiguousarray(ju[s::S]))
            return cache[s]
        per = int(np.ceil(iu.size / S))
        desc = f"cells k % {S} == step*{world} + rank"
    return slice_of, max(per, 1), desc, iu.size


# ------------------------------------------------------------------ main
def main():
    a = parse()
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(a))
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
    eng = (CpuStubEngine if a.cpu_stub else GpuEngine)(a, cfg, rank, world, local)
    shapes = np.array([eng.ds.shape(i) for i in range(a.n)], dtype=np.float64)

    S = a.slices
    if a.full:
        a.steps, a.warmup = 1, 0
    # the configured step size whatever --steps is: past S / N steps the slices
    # repeat (each step recomputed in full, as C2's whole-Gram steps repeat),
    # rather than shrinking the step to (warmup + steps) * N slices
    S = -(-S // world) * world  # a multiple of N: rank r's slices are cells k % N == r
    slice_of, per, step_kind, n_cells = make_plan(kind, a.n, world, rank, S)
    eng.alloc(per)

    def run_step(step):
        if a.full:  # the product path: sk_gram_sharded over all ranks
            from stem_kernel_amd import shard
            tm = eng.full()
            x, y = shard.rank_pairs(a.n, world, rank)
            return x, y, tm
        x, y = slice_of(step)
        return x, y, eng.step(x, y)

    # the steps' cell lists are host bookkeeping: formed before the timed region
    if not a.full:
        for t in range(a.warmup + a.steps):
            slice_of(t)
        if a.cpu_stub:
            for r in range(world):
                slice_of(a.warmup + a.steps - 1, r)
    if rank == 0:  # a line on stderr every minute: a long run is visibly alive
        import threading

        def heartbeat(t_start=time.perf_counter()):
            while True:
                time.sleep(60)
                print(f"[bench] running, {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
        threading.Thread(target=heartbeat, daemon=True).start()
    for w in range(a.warmup):
        run_step(w)
    eng.sync()
    if getattr(eng, "async_on", False):
        eng.totals()  # (the warmup's timings, dropped)
    eng.barrier()
    eng.sync()
    t0 = time.perf_counter()
    local_pairs = 0
    k_ms, work, cells, launches, l_ms = [], [], [], [], []

    def add(tm):
        k_ms.append(tm["stem_ms"])
        cells.append(tm["cells"])
        launches.append(tm["launches"])
        l_ms.append(tm["ms_sum"])
    for k in range(a.steps):
        x, y, tm = run_step(a.warmup + k)
        local_pairs += x.size
        if tm is not None:
            add(tm)
        work.append((x, y))
    eng.sync()
    eng.barrier()
    eng.sync()
    elapsed = time.perf_counter() - t0
    if getattr(eng, "async_on", False):  # every timed call's events, summed (outside the timed region)
        add(eng.totals())
        cells = [cells[0] / a.steps] * a.steps
    if eng.dist_on:
        elapsed, total_pairs = eng.reduce_max_sum(elapsed, local_pairs)
    else:
        total_pairs = float(local_pairs)
    if a.cpu_stub:
        last = a.warmup + a.steps - 1
        eng.verify(lambda r: slice_of(last, r))

    if rank == 0:
        value = total_pairs / elapsed
        xs = np.concatenate([w[0] for w in work])
        ys = np.concatenate([w[1] for w in work])
        # dominant kernel (stem / 4-D / BPLA): each launch timed by HIP events
        # around it on its own stream (sk_last_launch_ms), the launches' span
        # by sk_last_timing
        rf = None
        if not a.cpu_stub:
            rt = None
            if kind in ("ss", "stem"):  # the DAG schedule's row transfers per example (packed set)
                rt = np.array([list(eng.ds.row_traffic(i).values()) for i in range(a.n)], dtype=np.float64)
            rf = roofline(a.config, kind, a.length, shapes, xs, ys, float(np.sum(k_ms)), float(np.sum(l_ms)),
                          int(np.sum(launches)), cells, a.pmc_json, rt)
            rf["kernel"] = {"ss": "sk_dag_stem_kernel", "stem": "sk_dag_stem_kernel",
                            "stem4d": "sk_stem4d_kernel" if os.environ.get("SK4_NO_GSUM") else
                            "sk_stem4d_gsum_kernel" if os.environ.get("SK4_NO_PRE") else
                            "sk_stem4d_pre_kernel" if os.environ.get("SK4_SPAN") else "sk_stem4d_col_kernel",
                            "bpla": "sk_bpla_fast_kernel"}[kind]
        cpu, parity = None, None
        if not a.no_cpu_baseline and world == 1 and not a.cpu_stub:  # rank 0 at N=1 only
            cpu, cpairs, cvals, ccomp = cpu_baseline(cfg, eng.data, a.cpu_pairs)
            # the baseline's oracle values double as a parity check of the
            # benched kernel classes on the same inputs (1e-6 relative): the
            # headline kernel, and each DP of a composition on its own
            cx = np.array([p[0] for p in cpairs], np.int32)
            cy = np.array([p[1] for p in cpairs], np.int32)

            def rel(got, ref):
                return float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)))
            err = rel(eng.ctx.pairs(eng.ds, eng.kern, cx, cy), cvals)
            parity = {"pairs": int(cx.size), "max_rel_err": err, "tol": 1e-6,
                      "ok": bool(err < 1e-6), "against": "C oracle (cpu_baseline sample)"}
            if ccomp:
                parity["components"] = {}
                for name, ck in components(eng.kern).items():
                    e = rel(eng.ctx.pairs(eng.ds, ck, cx, cy), ccomp[name])
                    parity["components"][name] = {
                        "kernel": type(ck).__name__, "max_rel_err": e,
                        "ref_range": [float(np.min(ccomp[name])), float(np.max(ccomp[name]))]}
                    parity["ok"] = parity["ok"] and bool(e < 1e-6)
                    parity["max_rel_err"] = max(parity["max_rel_err"], e)
        kdesc = {
            "ss": (cfg.get("cls") or "SuStemStrKernel") + "(alpha=0.2,beta=0.3,loop_gap=0.2,gap=0.8,band=10)",
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
            "data": ("cpu stub (test compute + gloo all-gather; not a measurement)" if a.cpu_stub else
                     "synthetic (splitmix64 ACGU sequences, Nussinov-Boltzmann bpp stand-in for "
                     "ViennaRNA; no checkpoints)"),
            "config": {
                "workload": f"{a.config}: {a.n}x{a.n} {kdesc} Gram, L={cfg['L']}, "
                            f"step = 1/{S} of the {n_cells} upper-triangle pairs per GPU",
                "step_cells": step_kind,
                "n_sequences": a.n, "length": cfg["L"], "pairs_per_step_per_gpu": per,
                "kernel": kdesc, "basepair_th": 0.01,
                "cli_mode": {"ns": "stem_kernel_lite --log (LSuStemStrKernel, main.cpp:187-191); the CLI's "
                                   "plain SuStemStrKernel default only estimates memory (main.cpp:180-186)",
                             "c2": "ss_kernel.h StemStrKernel (SuStemStr sum; the --log mode costs the same)",
                             "c5": "stem_kernel_lite --no-string (SuStemKernel, main.cpp:193-198)",
                             "c3": "stem_kernel (4-D) default -p BPMatrix full_dp",
                             "c4": "bpla_kernel default"}[a.config],
                "parallelism": f"cyclic cell plan x{world} (sk_comm_allgather, RCCL)"
                               + (" -- full Gram via sk_gram_sharded" if a.full else ""),
                "mean_nodes": float(shapes[:, 0].mean()), "mean_edges": float(shapes[:, 1].mean()),
                "mean_bpfreq": float(shapes[:, 2].mean()),
                "host_build_s": round(eng.t_build, 2), "upload_s": round(eng.t_upload, 3),
            },
            "roofline": rf,
            "cpu_baseline": cpu,
            "parity": parity,
            "cells_per_step": float(np.mean(cells)),
        }
        if a.cpu_stub:
            line["stub_checked_pairs"] = eng.checked
        print(json.dumps(line), flush=True)
        if parity is not None and not parity["ok"]:
            print(f"PARITY FAILURE: max relative error {parity['max_rel_err']:.3g} > 1e-6",
                  file=sys.stderr, flush=True)
            sys.exit(3)
    eng.close()


if __name__ == "__main__":
    main()
