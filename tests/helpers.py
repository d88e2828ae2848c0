"""Shared test inputs: seeded sequences/alignments and their oracle twins."""
import numpy as np

import stem_kernel_amd as ska
from oracle import pyoracle as po


def make_examples(seqs_or_alns, th=0.01, use_bp=True):
    """Build the same examples in the product Dataset and the oracle."""
    ds = ska.Dataset()
    om = []
    for k, ex in enumerate(seqs_or_alns):
        rows = [ex] if isinstance(ex, str) else list(ex)
        bpps = [ska.fold(r.replace("-", "").lower()) for r in rows] if use_bp else None
        ds.add("+1" if k % 2 == 0 else "-1", rows, bpps, th=th, use_bp=use_bp)
        om.append(po.OMData(rows, bpps, th, use_bp))
    return ds, om


def mutate_alignment(seq, n_rows, seed, sub=0.1, gap=0.05):
    """Rows derived from seq with point substitutions and gap columns
    (SURVEY.md §8d, C4 generator)."""
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n_rows):
        r = list(seq)
        for i in range(len(r)):
            u = rng.random()
            if u < gap:
                r[i] = "-"
            elif u < gap + sub:
                r[i] = "ACGU"[rng.integers(4)]
        rows.append("".join(r))
    return rows


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))
