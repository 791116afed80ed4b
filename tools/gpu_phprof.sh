#!/bin/bash
# per-kernel statistics of the phase route at W windows (default 256)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export VIO_BA_PHASES=1
W=${W:-256}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ph$W -o ph --output-format csv -- python3 tools/ba_batch_run.py $W 10 > gpurun_out/prof_ph$W.log 2>&1 || exit 1
python3 - <<PY
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_ph$W/ph_kernel_stats.csv")))
for r in rows[:10]:
    print("W=$W %-40s calls %6s avg_us %9.2f" % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))
PY
