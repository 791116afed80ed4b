#!/bin/bash
# tracker: GPU parity tests, config-1 stage times, rocprofv3 kernel trace of the config-1 pipeline
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tracker_gpu.py tests/test_frontend_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_trk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_trk.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python3 tools/trk_time.py 20 > gpurun_out/trk_time.log 2>&1 || exit 1
cat gpurun_out/trk_time.log
rm -rf gpurun_out/trkprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trkprof -o trk --output-format csv -- python3 tools/trk_time.py 5 > gpurun_out/trk_prof.log 2>&1 || exit 1
echo prof ok
