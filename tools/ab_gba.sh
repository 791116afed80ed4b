#!/bin/bash
# Same-box A/B of global-BA library builds (VIO360_LIB): per round each library's per-iteration time
# (tools/gba_time.py), then per library the kernel statistics of a 3-iteration solve.  Usage: tools/ab_gba.sh <tag> <lib>...
set -u
tag=$1; shift
out=gpurun_out/abg_$tag
mkdir -p $out
export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
  for lib in "$@"; do
    VIO360_LIB=$lib timeout -k 10 200 python3 tools/gba_time.py 8 3 > $out/t.log 2>&1 || { echo "$lib failed"; tail -5 $out/t.log; exit 1; }
    echo "r$r $(basename $lib) $(tail -1 $out/t.log)"
  done
done
if [ "${STATS:-1}" = "1" ]; then
  for lib in "$@"; do
    n=$(basename $lib .so)
    VIO360_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks_$n -o run --output-format csv -- python3 tools/gba_run.py 3 > $out/ks_$n.log 2>&1 || { echo "stats $n failed"; exit 1; }
    f=$(find $out/ks_$n -name "*kernel_stats.csv" | head -1)
    echo "== $n"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'  {r["Name"][:60]:60s} n={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.2f} us tot={float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
  done
fi
