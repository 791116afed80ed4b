"""Timeline of the last tracker pipeline run in a rocprofv3 kernel trace (tools/gpu_prof.sh / tools/ab_trk.sh output):
start / end of every kernel relative to the run's first pyr_down launch.
usage: python tools/trk_timeline.py gpurun_out/prof_<tag>/run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "pyr_down" in r["Kernel_Name"] or "pyr3_kernel" in r["Kernel_Name"]]
s = idx[-1] if "pyr3_kernel" in rows[idx[-1]]["Kernel_Name"] else idx[-3]
t0 = int(rows[s]["Start_Timestamp"])
for r in rows[s:s + 24]:
    n = r["Kernel_Name"].split("(")[0].replace("vio360::", "")[:40]
    a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{n:40s} q={r['Queue_Id']:>3s} start={a / 1e3:8.2f} end={b / 1e3:8.2f} dur={(b - a) / 1e3:7.2f}")
