#!/bin/bash
# full GPU suite, BA timings, tracker stage times + kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/ba_quick.py > gpurun_out/ba_quick.log 2>&1 || exit 1
grep -E "windows=|cfg3" gpurun_out/ba_quick.log
timeout -k 10 120 python3 tools/trk_time.py 20 > gpurun_out/trk_time.log 2>&1 || exit 1
cat gpurun_out/trk_time.log
rm -rf gpurun_out/trkprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trkprof -o trk --output-format csv -- python3 tools/trk_time.py 5 > gpurun_out/trk_prof.log 2>&1 || exit 1
echo prof ok
