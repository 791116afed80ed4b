#!/bin/bash
# per-kernel stats of the phase route (tools/ba_batch_run.py W 20) for each library: args W lib...
set -u
export TMPDIR=/tmp VIO_BA_PHASES=1
W=$1; shift
for lib in "$@"; do
  b=$(basename $lib .so); d=gpurun_out/abst_${b}_$W
  rm -rf $d
  VIO360_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/ba_batch_run.py $W 20 > $d.log 2>&1 || exit 1
  echo "== $b W=$W"
  python3 - $(find $d -name "*kernel_stats.csv" | head -1) <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "ph_" in r["Name"]:
        print(f"  {r['Name'].split('(')[0].replace('vio360::','')[:34]:34s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
done
