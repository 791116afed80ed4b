#!/bin/bash
# HBM traffic of the BA phase route at the config-4 shard (256 windows x 10 iterations, default route):
# one rocprofv3 PMC pass per counter over tools/ba_batch_run.py.  Summary: tools/pmc_summary.py.
set -u
mkdir -p gpurun_out/pmc_ba
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_ba/$ctr
  timeout -k 10 240 rocprofv3 --pmc $ctr -d gpurun_out/pmc_ba/$ctr -o run --output-format csv -- \
      python3 tools/ba_batch_run.py 256 3 > gpurun_out/pmc_ba/$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc"; tail -1 gpurun_out/pmc_ba/$ctr.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_ba gpurun_out/pmc_ba/traffic.json
