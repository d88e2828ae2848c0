"""Generate tests/golden/large_*.npz: oracle values at the benchmark
configurations' sizes, so the GPU parity suite reaches every kernel
instantiation the benches run.

Which instantiation runs depends on the input size:

* DAG stem kernel (stem_kernel_lite/stem_kernel.cpp:14-95): one register
  class per y example, MAXK = 64-node slots per lane = ceil(non-leaf
  nodes / 64) rounded up to 4, except 17 slots (1,025-1,088 nodes: its own
  class since r06).  C2 (L=150) runs MAXK 16, NS (L=200) 16/17/20,
  C5 (L=300) 20/24/28; the L=380/420 examples add 28/32 (2,047 nodes, the
  kernel's limit).  The profile string kernel runs 3-7 strips of 64 rows.
* 4-D stem kernel full_dp (stem_kernel/stem_kernel.cpp:282-351): CPL = cells
  per lane = 4 for |y| < 256 (C3, L=200), 8 for 256 <= |y| < 512; banded
  partial_dp (:113-280) is a separate instantiation.
* BPLA (bpla_kernel/bpla_kernel.cpp:64-115, 159-174): C4's 4-row alignments
  of L 190-210 (bench.py's generator), 4 strips.

Inputs are the first examples of the benches' own seeded sets (bench.py
CONFIGS, seed 0x5EED0000 + config id), stored verbatim; base-pairing
probabilities are the engine's synthetic fold (stem_kernel_amd.fold, host
C++), whose bytes are pinned by a SHA-256 stored beside the values.
Expected values come from the CPU oracle (oracle/sk_oracle.c), a line-by-line
restatement of the reference (parity against the reference's own output is
unpinned: it ships no fixtures and its DP does not build here).

Run:  python tests/golden/make_golden_large.py [--dag-only]     (~1-2 min on 8 cores)
"""
import hashlib
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import stem_kernel_amd as ska  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

DAG_KINDS = (0, 1, 2, 3)  # SuStem, SiStem, SuStr, SiStr (4, 5 are their sums)
BPLA_KINDS = (9, 10, 11, 12)


def fold_rows(rows):
    return [ska.fold(r.replace("-", "").lower()) for r in rows]


def bpp_digest(examples):
    h = hashlib.sha256()
    for rows in examples:
        for b in fold_rows(rows):
            h.update(np.ascontiguousarray(b, np.float64).tobytes())
    return h.hexdigest()


def dag_sets():
    """name -> list of single-sequence examples."""
    out = {
        "c2_L150": ska.random_sequences(6, 150, 0x5EED0001),
        "ns_L200": ska.random_sequences(6, 200, 0x5EED0002),
        "c5_L300": ska.random_sequences(6, 300, 0x5EED0004),
    }
    # the widest classes: examples of 1,537-2,048 non-leaf nodes
    wide = []
    for L, seed in ((380, 0x5EED0104), (420, 0x5EED0105)):
        for s in ska.random_sequences(12, L, seed):
            ds = ska.Dataset.synthetic([s])
            nl = int(np.sum(ds.dag(0)["n_edges"] > 0))
            if nl <= 2048 and len([w for w in wide if len(w) == L]) < 2 and \
                    (L == 380 or nl > 1792):
                wide.append(s)
    out["wide_L380_420"] = wide
    # NS-size y of 1,089-1,280 non-leaf nodes (the MAXK 20 class, since r06's
    # MAXK 17 class takes 1,025-1,088): the first three such examples of the
    # NS stream past the six above
    ns20 = []
    for s in ska.random_sequences(64, 200, 0x5EED0002)[6:]:
        ds = ska.Dataset.synthetic([s])
        nl = int(np.sum(ds.dag(0)["n_edges"] > 0))
        if 1088 < nl <= 1280 and len(ns20) < 3:
            ns20.append(s)
    out["ns20_L200"] = ns20
    # ... and of 896-958 (MAXK 16's lower end; r06k measured 12-wave classes
    # of 13-15 slots for them, not shipped): the first two such
    ns15 = []
    for s in ska.random_sequences(64, 200, 0x5EED0002)[6:]:
        ds = ska.Dataset.synthetic([s])
        nl = int(np.sum(ds.dag(0)["n_edges"] > 0))
        if 896 <= nl <= 958 and len(ns15) < 2:
            ns15.append(s)
    out["ns15_L200"] = ns15
    return out


_OM = {}


def _dag_cell(args):
    name, seqs, kind, i, j = args
    key = name
    if key not in _OM:
        _OM[key] = [po.OMData([s], [ska.fold(s.lower())], 0.01) for s in seqs]
    om = _OM[key]
    p = ska.SuStemStrKernel().params
    return po.kernel_value(kind, om[i], om[j], p)


def _s4d_cell(args):
    a, b, band = args
    return po.stem4d(a.lower(), ska.fold(a.lower()), b.lower(), ska.fold(b.lower()),
                     float(np.float32(0.8)), 1.0, 0.5, 0.0, 0, 3, band)


_BOM = {}


def _bpla_cell(args):
    alns, kind, i, j = args
    if not _BOM:
        for k, rows in enumerate(alns):
            _BOM[k] = po.OMData(rows, fold_rows(rows), 0.01)
    p = ska.BPLAKernel().params
    return po.kernel_value(kind, _BOM[i], _BOM[j], p)


def main():
    jobs = min(8, os.cpu_count() or 1)
    arrays = {}
    with ProcessPoolExecutor(jobs) as ex:
        for name, seqs in dag_sets().items():
            n = len(seqs)
            arrays[f"{name}_seqs"] = np.array(seqs)
            arrays[f"{name}_sha"] = np.array(bpp_digest([[s.lower()] for s in seqs]))
            for kind in DAG_KINDS:
                cells = [(name, seqs, kind, i, j) for i in range(n) for j in range(n)]
                v = np.array(list(ex.map(_dag_cell, cells, chunksize=1))).reshape(n, n)
                arrays[f"{name}_K{kind}"] = v
            print(name, n, "examples, L =", sorted({len(s) for s in seqs}), flush=True)
    np.savez_compressed(os.path.join(HERE, "large_dag.npz"), **arrays)
    if "--dag-only" in sys.argv:
        return

    # 4-D full_dp at C3's L=200 (CPL 4), CPL 8 at |y| = 260, banded partial_dp
    c3 = ska.random_sequences(3, 200, 0x5EED0002)
    long_ = ska.random_sequences(1, 260, 0x5EED0202)[0]
    cases = [(c3[0], c3[1], 0), (c3[2], c3[0], 0), (c3[1], c3[1], 0), (c3[0], long_, 0),
             (c3[1], c3[2], 10)]
    with ProcessPoolExecutor(jobs) as ex:
        vals = list(ex.map(_s4d_cell, cases))
    np.savez_compressed(os.path.join(HERE, "large_4d.npz"),
                        x=np.array([c[0] for c in cases]), y=np.array([c[1] for c in cases]),
                        band=np.array([c[2] for c in cases], np.int32), value=np.array(vals),
                        sha=np.array(bpp_digest([[c[0].lower()] for c in cases] +
                                                [[c[1].lower()] for c in cases])))
    print("4-D", len(cases), "pairs", flush=True)

    # BPLA: the first alignments of bench.py's C4 set (4 rows, L 190-210)
    import bench
    alns = bench.c4_alignments(2048, 190, 210, 4, 0x5EED0003)[:6]
    n = len(alns)
    arrays = {"rows": np.array([r for a in alns for r in a]), "n_rows": np.array([4] * n),
              "sha": np.array(bpp_digest(alns))}
    with ProcessPoolExecutor(jobs) as ex:
        for kind in BPLA_KINDS:
            cells = [(alns, kind, i, j) for i in range(n) for j in range(n)]
            arrays[f"K{kind}"] = np.array(list(ex.map(_bpla_cell, cells))).reshape(n, n)
    np.savez_compressed(os.path.join(HERE, "large_bpla.npz"), **arrays)
    print("BPLA", n, "alignments", flush=True)


if __name__ == "__main__":
    main()
