"""Per-kernel mean of every counter in a rocprofv3 PMC output directory (diagnostic print).

usage: python tools/pmc_counters.py <rocprofv3 -d directory> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(src, pat=""):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("vio360::", "")
                if pat in k:
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(vals):
        cs = vals[k]
        n = max(len(v) for v in cs.values())
        print(k, "dispatches", n, " ".join(f"{c}={sum(v) / len(v):.0f}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main(*sys.argv[1:])
