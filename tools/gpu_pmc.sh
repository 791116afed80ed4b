#!/bin/bash
# HBM traffic of the hot kernels: rocprofv3 PMC passes, one counter group per pass (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950; no tracing domains with --pmc on this pool).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $ctr -d gpurun_out/pmc/$ctr -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --klt-steps 5 > gpurun_out/pmc/$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
