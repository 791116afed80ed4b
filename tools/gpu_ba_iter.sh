#!/bin/bash
# BA iteration loop: GPU BA parity tests, route timings at 256 windows and 1 window, phase-route trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/route_ab.log
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_ba.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in VIO_BA_PHASES VIO_BA_MONOLITHIC; do
  env $r=1 timeout -k 10 120 python3 tools/ba_batch_run.py 256 10 >> gpurun_out/route_ab.log 2>&1 || exit 1
done
VIO_BA_PHASES=1 timeout -k 10 120 python3 tools/ba_batch_run.py 1 20 >> gpurun_out/route_ab.log 2>&1 || exit 1
grep W= gpurun_out/route_ab.log
bash tools/gpu_phtrace.sh && head -12 gpurun_out/prof_ph256/ph_kernel_stats.csv | cut -d, -f1-4
