#!/bin/bash
# tracker A/B on one box: per round the config-1 pipeline time (tools/trk_time.py) with each setting of an
# environment variable (AB_VAR; values in AB_VALS), then the kernel trace timeline of the last value.
set -u
tag=$1
out=gpurun_out/abt_$tag
mkdir -p $out
export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-3}); do
  for v in $AB_VALS; do
    env $AB_VAR=$v timeout -k 10 120 python3 tools/trk_time.py 30 > $out/t.log 2>&1 || { echo "$AB_VAR=$v failed"; tail -5 $out/t.log; exit 1; }
    echo "r$r $AB_VAR=$v $(grep total_ms $out/t.log)"
  done
done
if [ "${TIMELINE:-1}" = "1" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python3 tools/trk_time.py 10 > $out/trace.log 2>&1 || { echo trace failed; exit 1; }
  f=$(find $out/trace -name "*kernel_trace.csv" | head -1)
  python3 tools/trk_timeline.py $f | head -20
  rm -rf $out/trace
fi
