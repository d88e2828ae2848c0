"""Kernel statistics (rocprofv3 --stats CSV columns) from a rocprofv3 rocpd
SQLite output (a run made without --output-format csv)."""
import math
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    t = {r[0].split("_0")[0]: r[0] for r in c.execute("select name from sqlite_master where type='table'")}
    rows = c.execute(f"select s.display_name, d.end - d.start from {t['rocpd_kernel_dispatch']} d "
                     f"join {t['rocpd_info_kernel_symbol']} s on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dur in rows:
        agg.setdefault(name, []).append(dur)
    tot = sum(sum(v) for v in agg.values())
    with open(out, "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n')
        for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            n, s = len(v), sum(v)
            avg = s / n
            sd = math.sqrt(sum((x - avg) ** 2 for x in v) / n)
            f.write(f'"{name}",{n},{s},{avg:.6f},{100.0 * s / tot:.2f},{min(v)},{max(v)},{sd:.6f}\n')


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
