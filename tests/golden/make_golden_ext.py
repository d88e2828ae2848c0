"""Generate tests/golden/ext_small.npz: oracle vectors for the 4-D kernel's
-a alignment constraints (both LogValue zerop semantics) and for the BPLA
gradients (bpla_optimizer's per-pair step).

Produced by the CPU oracle (oracle/sk_oracle.c) like lite_small.npz: the
reference cannot be built here and ships no fixtures, so these pin the oracle
and the GPU engine against regressions ("parity unpinned" against the
reference's own output; the gradients are additionally pinned by finite
differences in tests/test_bpla_grad.py).

Run:  python tests/golden/make_golden_ext.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import stem_kernel_amd as ska  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from tests.helpers import mutate_alignment  # noqa: E402


def indel_variants(seed, n, L):
    rng = np.random.default_rng(seed)
    base = ska.random_sequences(1, L, seed)[0]
    out = [base]
    for _ in range(n - 1):
        r = []
        for c in base:
            u = rng.random()
            if u < 0.06:
                continue
            r.append("ACGU"[rng.integers(4)] if u < 0.2 else c)
            if rng.random() < 0.06:
                r.append("ACGU"[rng.integers(4)])
        out.append("".join(r))
    return out


def main():
    # -a constraints and partial_dp values (StemKernel4D defaults, bpp model 0)
    seqs = indel_variants(101, 4, 40)
    p4 = ska.StemKernel4D().params
    pairs = [(0, 1), (1, 0), (2, 3), (0, 3)]
    settings = [(0.5, 0, 1), (0.8, 3, 1), (0.5, 2, 0)]  # ali_bound, band, zerop_fixed
    lo, hi, val = [], [], []
    for ab, band, fixed in settings:
        for a, b in pairs:
            x, y = seqs[a].lower(), seqs[b].lower()
            l_, h_ = po.alignment_constraints(x, y, ab, band, fixed)
            lo.append(np.pad(l_.astype(np.int32), (0, 64 - l_.size), constant_values=-1))
            hi.append(np.pad(h_.astype(np.int32), (0, 64 - h_.size), constant_values=-1))
            val.append(po.stem4d(x, ska.fold(seqs[a]), y, ska.fold(seqs[b]), p4.gap, p4.stack,
                                 p4.subst, p4.bp_bound, p4.bp_model, p4.loop, band, ab, fixed))
    # BPLA gradients over small alignments
    alns = [mutate_alignment(s, 3, 200 + k) for k, s in enumerate(ska.random_sequences(3, 36, 0x5EED0203))]
    rows, ex_rows, bpps = [], [], []
    for a in alns:
        ex_rows.append(len(a))
        for r in a:
            rows.append(r)
            bpps.append(ska.fold(r.replace("-", "").lower()))
    om, k = [], 0
    for nr in ex_rows:
        om.append(po.OMData(rows[k:k + nr], bpps[k:k + nr], 0.01))
        k += nr
    pb = ska.BPLAKernel().params
    t = np.array(list(pb.score_table))
    gpairs = [(i, j) for i in range(len(om)) for j in range(i, len(om))]
    gv, gg = [], []
    for a, b in gpairs:
        v, d, _ = po.bpla_gradients(om[a], om[b], pb.alpha, pb.beta, pb.gap, pb.ext, t)
        gv.append(v)
        gg.append(d)
    np.savez_compressed(
        os.path.join(HERE, "ext_small.npz"),
        s4_seqs=np.array(seqs), s4_pairs=np.array(pairs, np.int32),
        s4_settings=np.array(settings, np.float64), s4_lo=np.array(lo), s4_hi=np.array(hi),
        s4_val=np.array(val),
        g_rows=np.array(rows), g_ex_rows=np.array(ex_rows, np.int32),
        g_pairs=np.array(gpairs, np.int32), g_val=np.array(gv), g_grad=np.array(gg))
    print("wrote ext_small.npz:", len(val), "constraint cases,", len(gv), "gradient pairs")


if __name__ == "__main__":
    main()
