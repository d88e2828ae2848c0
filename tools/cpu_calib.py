#!/usr/bin/env python3
"""Calibrate the CPU baseline's port against the reference's own DAG stem DP.

BASELINE.md's probe timed the reference's stem_kernel_lite/stem_kernel.cpp:
14-95 itself (compiled in this container against stand-in headers, which is
allowed for a probe but not for an oracle) at 57 ms per pair, L = 200, one
core, on synthetic Nussinov-Boltzmann bpp.  This script times the port (the
C oracle, oracle/sk_oracle.c, the bench's cpu_baseline) on the same kind of
pairs on one core of the same container and writes the ratio to
profiles/r04_cpu_calibration.json; bench.py reports it beside its baseline
(cpu_baseline.calibration).  Test infrastructure only."""
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    import stem_kernel_amd as ska
    from oracle import pyoracle as po
    seqs = ska.random_sequences(64, 200, 0x5EED0002)
    om = [po.OMData([s], [ska.fold(s)], 0.01) for s in seqs]
    p = ska.SuStemKernel().params
    rng = np.random.default_rng(1)
    pairs = [tuple(sorted(int(v) for v in rng.choice(64, 2, replace=False))) for _ in range(200)]
    reps = []
    for _ in range(3):  # the container's cores are shared: median of three
        t = time.perf_counter()
        for a, b in pairs:
            po.kernel_value(0, om[a], om[b], p)
        reps.append((time.perf_counter() - t) / len(pairs) * 1e3)
    port_ms = float(np.median(reps))
    ref_ms = 57.0  # reference DAG stem kernel, L=200, one core, this container
    out = {"what": "SuStemKernel at L=200 (th 0.01, band 10), one core, same container",
           "port_ms_per_pair": round(port_ms, 2), "port_pairs_per_s_per_core": round(1e3 / port_ms, 2),
           "reference_ms_per_pair": ref_ms, "reference_source": "BASELINE.md probe table (L=200 row)",
           "port_over_reference": round(ref_ms / port_ms, 3),
           "port_ms_per_pair_runs": [round(v, 2) for v in reps],
           "cpu_model": cpu_model(), "nproc": os.cpu_count(), "pairs": len(pairs)}
    path = os.path.join(ROOT, "profiles", "r04_cpu_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
