"""HBM bytes of one config-5 LM iteration from the PMC passes of tools/gpu_pmc_gba.sh: every dispatch's
FETCH_SIZE (x2, the gfx950 correction of wide coalesced reads, /opt/skills/guides/MI355X_MICROARCH.md)
and WRITE_SIZE (KB), summed per run; per iteration = (3-iteration run - 1-iteration run) / 2.
Output JSON: hbm_bytes_per_iteration (bench.py global_ba.roofline.traffic) and the per-kernel split.

usage: python tools/pmc_gba_summary.py gpurun_out/pmc_gba profiles/r3_pmc_traffic_gba.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def sums(pass_dir, counter):
    tot = defaultdict(float)
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter:
                    name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                    tot[name.replace("void ", "").replace("vio360::", "").strip()] += float(row["Counter_Value"]) * 1024.0
    return tot


def main(src, dst):
    runs = {}
    for n in (1, 3):
        rd = sums(os.path.join(src, f"n{n}", "FETCH_SIZE"), "FETCH_SIZE")
        wr = sums(os.path.join(src, f"n{n}", "WRITE_SIZE"), "WRITE_SIZE")
        runs[n] = {k: (2.0 * rd.get(k, 0.0), wr.get(k, 0.0)) for k in set(rd) | set(wr)}
    per = {}
    for k in set(runs[1]) | set(runs[3]):
        a, b = runs[3].get(k, (0.0, 0.0)), runs[1].get(k, (0.0, 0.0))
        per[k] = {"read_bytes": (a[0] - b[0]) / 2.0, "write_bytes": (a[1] - b[1]) / 2.0}
    total = sum(v["read_bytes"] + v["write_bytes"] for v in per.values())
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, 1- and 3-iteration "
                     "config-5 solves (tools/gpu_prof.sh gba)",
           "correction": "reads = 2 x FETCH_SIZE (gfx950 half-count of wide coalesced reads), writes as reported",
           "hbm_bytes_per_iteration": total,
           "kernels_per_iteration": dict(sorted(per.items(), key=lambda kv: -(kv[1]["read_bytes"] + kv[1]["write_bytes"])))}
    if os.environ.get("VIO_COMMIT"):  # the profiled build (tools/gpu_prof.sh); bench.py reports it with the traffic
        doc["commit"] = os.environ["VIO_COMMIT"]
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"HBM bytes per LM iteration: {total / 1e9:.3f} GB")
    for k, v in list(doc["kernels_per_iteration"].items())[:12]:
        print(f"  {k:50s} rd {v['read_bytes'] / 1e6:10.1f} MB  wr {v['write_bytes'] / 1e6:10.1f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
