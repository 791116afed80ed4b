#!/bin/bash
# per-kernel statistics of the phase route, one workload per rocprofv3 run (isolated per batch size):
# W windows x 10 fixed LM iterations, S solves (tools/ba_batch_run.py)
set -u
tag=${1:-r3}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$tag
for cfg in "1 20" "32 10" "256 5"; do
  set -- $cfg
  d=gpurun_out/prof_$tag/w$1
  rm -rf $d
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/ba_batch_run.py $1 $2 > $d.log 2>&1
  rc=$?; echo "W=$1 rc=$rc $(tail -1 $d.log | cut -c1-160)"
  if [ $rc -ne 0 ]; then exit $rc; fi
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$1" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "ph_" in n or "ba_" in n:
        print(f"  W={sys.argv[2]} {n.split('(')[0].replace('vio360::',''):40s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.2f} min_us={float(r['MinNs'])/1e3:8.2f}")
PY
done
