#!/bin/bash
# kernel statistics of the 256-window shard (phase route) and the 32-window shard: rocprofv3 --kernel-trace --stats
set -u
tag=${1:-x}
out=gpurun_out/ks_$tag
mkdir -p $out
export TMPDIR=/tmp
for W in 256 32; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/ks_$W -o run --output-format csv -- python3 tools/ba_batch_run.py $W 10 > $out/ks_$W.log 2>&1 || { echo "ks_$W failed"; tail -3 $out/ks_$W.log; exit 1; }
  tail -1 $out/ks_$W.log | cut -c1-200
done
