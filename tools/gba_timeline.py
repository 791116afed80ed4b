"""Timeline of global-BA Cholesky kernels from a rocprofv3 kernel trace (a window of consecutive launches
from the middle of the run): queue, start / end relative to the first, grid.
usage: python tools/gba_timeline.py <kernel_trace.csv> [first] [count]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ch = [r for r in rows if "chol_" in r["Kernel_Name"] or "trsv" in r["Kernel_Name"]]
a = int(sys.argv[2]) if len(sys.argv) > 2 else len(ch) // 3
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
t0 = int(ch[a]["Start_Timestamp"])
for r in ch[a:a + n]:
    nm = r["Kernel_Name"].split("(")[0].replace("vio360::", "")
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{nm:28s} q={r['Queue_Id']:>2s} s={s / 1e3:9.2f} e={e / 1e3:9.2f} dur={(e - s) / 1e3:7.2f} grid={r['Grid_Size_X']}")
