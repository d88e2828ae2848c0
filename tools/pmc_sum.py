"""Sum rocprofv3 --pmc counter CSVs per kernel (substring match).
    python tools/pmc_sum.py DIR KERNEL_SUBSTRING  -> JSON {counter: total, dispatches: n}"""
import csv
import glob
import json
import os
import sys


def main(d, sub):
    tot, disp = {}, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if sub not in r.get("Kernel_Name", ""):
                    continue
                disp.add((f, r.get("Dispatch_Id")))
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    tot["dispatches"] = len(disp)
    print(json.dumps(tot))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
