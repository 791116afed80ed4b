#!/bin/bash
# Tracker parity tests + a KLT-only bench line with the rocprof kernel summary.  Stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tracker_gpu.py tests/test_frontend_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_trk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_trk.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trk -o trk --output-format csv -- python3 bench.py --steps 2 --warmup 1 --windows 8 --no-cpu-baseline --no-global --klt-steps 20 > gpurun_out/bench_trk.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/bench_trk.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['erp_klt']))"
exit $rc
