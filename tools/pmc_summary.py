"""Median per-dispatch value of every counter in rocprofv3 --pmc output directories, per kernel
(substring match on the demangled name). Usage: pmc_summary.py KERNEL_SUBSTR DIR [DIR ...]"""
import csv
import glob
import os
import statistics
import sys


def collect(d, kern):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kern not in row.get("Kernel_Name", ""):
                continue
            key = (row["Counter_Name"], row["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (c, _), v in vals.items():
        out.setdefault(c, []).append(v)
    return {c: statistics.median(v) for c, v in out.items()}


if __name__ == "__main__":
    kern = sys.argv[1]
    res = {}
    for d in sys.argv[2:]:
        res.update(collect(d, kern))
    for k in sorted(res):
        print(f"{k:28s} {res[k]:16.1f}")
