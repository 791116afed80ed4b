#!/bin/bash
# tracker: bitwise GPU tests, stage times, per-kernel stats of the config-1 pipeline
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-trk7}
timeout -k 10 300 python -u -m pytest tests/test_tracker_gpu.py tests/test_frontend_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; fi
timeout -k 10 120 python3 tools/trk_time.py 30 > gpurun_out/trk_$tag.log 2>&1 || exit $?
grep -E "total|ransac|gftt|lk|pyr" gpurun_out/trk_$tag.log | head
d=gpurun_out/prof_$tag
rm -rf $d
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/trk_time.py 30 > $d.log 2>&1 || exit $?
f=$(find $d -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("vio360::", "")
    print(f"  {n[:60]:60s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.2f} min_us={float(r['MinNs'])/1e3:8.2f}")
PY
