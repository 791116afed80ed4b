"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; tools/gpu_pmc.sh).

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch.  The gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) is applied to reads: FETCH_SIZE reports half
of the bytes of wide coalesced reads, so the read bytes are 2 x FETCH_SIZE x 1024.  Writes are taken
as reported.  Output: JSON {kernel: {dispatches, read_bytes_per_launch, write_bytes_per_launch,
hbm_bytes_per_launch, fetch_kb_raw, write_kb_raw}} — bench.py reads it for the roofline `traffic`.

usage: python tools/pmc_summary.py gpurun_out/pmc profiles/r1_pmc_traffic.json
The commit the profiled tree was built from goes into the summary's "commit" field (VIO_COMMIT, else
`git rev-parse HEAD` where a checkout exists): bench.py reports it next to the traffic figure.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pass_dir, counter):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def short(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("void ", "").replace("vio360::", "").strip()


def main(src, dst):
    fetch = load(os.path.join(src, "FETCH_SIZE"), "FETCH_SIZE")
    write = load(os.path.join(src, "WRITE_SIZE"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        n = max(len(f), len(w))
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        rd = 2.0 * fk * 1024.0
        wr = wk * 1024.0
        key = short(k)
        if key in out:  # template instances etc.: keep the most dispatched
            if out[key]["dispatches"] >= n:
                continue
        out[key] = {"dispatches": n, "fetch_kb_raw": fk, "write_kb_raw": wk, "read_bytes_per_launch": rd,
                    "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr}
    commit = os.environ.get("VIO_COMMIT")
    if not commit:
        import subprocess
        try:
            commit = subprocess.run(["git", "rev-parse", "HEAD"], capture_output=True, text=True,
                                    cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip() or None
        except OSError:
            commit = None
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/gpu_pmc.sh)",
           "commit": commit,
           "correction": "reads = 2 x FETCH_SIZE (gfx950 half-count of wide coalesced reads), writes as reported",
           "kernels": out}
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches"])[:25]:
        print(f"{k:60s} n={v['dispatches']:5d} rd/launch={v['read_bytes_per_launch'] / 1e6:10.3f} MB "
              f"wr/launch={v['write_bytes_per_launch'] / 1e6:10.3f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
