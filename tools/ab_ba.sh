#!/bin/bash
# Same-box A/B of window-BA library builds: for each round, each library in turn (VIO360_LIB), the resident
# batch time at the given window counts (tools/ba_batch_run.py), then per library one rocprofv3 --stats run at
# 256 windows (per-kernel averages).  Usage: tools/ab_ba.sh <tag> <lib>... ; WINDOWS / ROUNDS env.  A library
# argument may carry one environment setting for its runs: <lib>@VAR=VALUE.
set -u
tag=$1; shift
out=gpurun_out/ab_$tag
mkdir -p $out
export TMPDIR=/tmp
WINDOWS=${WINDOWS:-"1 32 256"}
ROUNDS=${ROUNDS:-3}
for r in $(seq $ROUNDS); do
  for arg in "$@"; do
    lib=${arg%%@*}; ev=VIO_AB_NONE=1; [ "$arg" != "$lib" ] && ev=${arg#*@}
    for W in $WINDOWS; do
      env $ev VIO360_LIB=$lib timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 > $out/run.log 2>&1 || { echo "$arg W=$W failed"; tail -5 $out/run.log; exit 1; }
      echo "r$r $(basename $arg) $(tail -1 $out/run.log)"
    done
  done
done
if [ "${STATS:-1}" = "1" ]; then
  for arg in "$@"; do
    lib=${arg%%@*}; n=$(basename "$arg" | tr '@=' '__'); ev=VIO_AB_NONE=1; [ "$arg" != "$lib" ] && ev=${arg#*@}
    env $ev VIO360_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/ks_$n -o run --output-format csv -- python3 tools/ba_batch_run.py 256 10 > $out/ks_$n.log 2>&1 || { echo "stats $n failed"; exit 1; }
    f=$(find $out/ks_$n -name "*kernel_stats.csv" | head -1)
    echo "== $n"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'  {r["Name"][:60]:60s} n={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.2f} us')
PY
  done
fi
