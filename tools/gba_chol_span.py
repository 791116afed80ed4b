"""Per-LM-iteration span of the Cholesky + triangular solves in a rocprofv3 kernel trace (first chol_ /
trsv launch to the last, launches more than 300 us apart start a new iteration).
usage: python tools/gba_chol_span.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted((r for r in csv.DictReader(open(sys.argv[1])) if "chol_" in r["Kernel_Name"] or "trsv" in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
spans, s0, e0 = [], None, None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s0 is None or s - e0 > 300000:
        if s0 is not None:
            spans.append((e0 - s0) / 1e6)
        s0, e0 = s, e
    e0 = max(e0, e)
spans.append((e0 - s0) / 1e6)
print("Cholesky + solves per LM iteration (ms):", " ".join(f"{x:.3f}" for x in spans),
      f"| median {sorted(spans)[len(spans) // 2]:.3f}")
