"""Throughput of the McCaskill fold (sk_fold_mccaskill, f1) against the CPU
oracle restatement (oracle/fold_oracle.c) on host threads.

    python tools/fold_bench.py [n_seqs] [length] [cpu_sample]
"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import stem_kernel_amd as ska  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ns = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    seqs = ska.random_sequences(n, L, 0x5EED0002)
    ctx = ska.Context(0)
    ctx.fold(seqs[:64])  # warm-up
    t = time.perf_counter()
    got = ctx.fold(seqs)
    gpu_s = time.perf_counter() - t
    threads = min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        ref = list(ex.map(lambda s: po.fold_mccaskill(s)[1], seqs[:ns]))
    cpu_s = time.perf_counter() - t
    err = max(float(np.max(np.abs(a - b))) for a, b in zip(got[:ns], ref))
    t = time.perf_counter()
    ds = ska.Dataset.folded(ctx, seqs)
    folded_s = time.perf_counter() - t
    print(json.dumps({"metric": f"McCaskill folds/s at L={L}", "n_seqs": n, "gpu_seq_per_s": n / gpu_s,
                      "gpu_s": gpu_s, "cpu_seq_per_s": ns / cpu_s, "cpu_threads": threads,
                      "cpu_sample": ns, "max_abs_err_vs_oracle": err,
                      "dataset_folded_seq_per_s": n / folded_s, "dataset_size": len(ds)}))


if __name__ == "__main__":
    main()
