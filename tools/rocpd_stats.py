"""rocprofv3 database (rocpd sqlite, the default output format) -> the
kernel stats CSV that `rocprofv3 --stats --output-format csv` writes
(Name, Calls, TotalDurationNs, AverageNs, Percentage).

    python tools/rocpd_stats.py gpurun_out/prof_c4/c4_results.db profiles/x_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels order by total_duration desc"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_ALL)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, calls, tot_us, avg_us, pct in rows:  # the view reports microseconds
            w.writerow([name, calls, round(tot_us * 1e3), f"{avg_us * 1e3:.3f}", f"{pct:.4f}"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
