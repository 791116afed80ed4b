"""Compare isolated kernel statistics (rocprofv3 --stats) of the window-BA kernels between two profiles:
ks_compare.py <old kernel_stats.csv> <new dir or csv>"""
import csv
import glob
import os
import sys


def rd(p):
    if os.path.isdir(p):
        p = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)[0]
    return {r["Name"][:40]: (float(r["AverageNs"]) / 1e3, int(r["Calls"])) for r in csv.DictReader(open(p))}


a, b = rd(sys.argv[1]), rd(sys.argv[2])
for k in b:
    if "ph_" in k or "cluster" in k:
        print(f"  {k:42s} {a.get(k, (0, 0))[0]:8.1f} {b[k][0]:8.1f} us  calls {b[k][1]}")
