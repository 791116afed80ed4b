#!/bin/bash
# tracker parity tests + a KLT-focused bench run + its rocprof kernel stats
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTEST_K="tracker or frontend or resize" bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --windows 8 --no-global --no-imu --no-tri --no-resize --no-config4 --no-cpu-baseline --klt-steps 20 > gpurun_out/bench_klt.log 2>&1
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_klt.log; exit $rc; fi
rm -rf gpurun_out/proft
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proft -o t --output-format csv -- python3 bench.py --steps 3 --warmup 1 --windows 8 --no-global --no-imu --no-tri --no-resize --no-config4 --no-cpu-baseline --klt-steps 20 > gpurun_out/proft.log 2>&1
echo "rocprof rc=$?"
