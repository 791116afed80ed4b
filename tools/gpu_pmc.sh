#!/bin/bash
# HBM traffic of the hot kernels: rocprofv3 PMC passes, one counter per pass (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950; no tracing domains with --pmc on this pool), over the
# default bench workload (BA batch + ERP-KLT pipeline).  Summary: tools/pmc_summary.py.
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc/$ctr
  timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/pmc/$ctr -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-global --klt-steps 5 --windows 256 --lm-iters 10 > gpurun_out/pmc/$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc"; tail -2 gpurun_out/pmc/$ctr.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/traffic.json
