#!/bin/bash
# global BA: triangular solves with data polling (tools/probe/libvio360_poll.so) vs the in-tree library
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
VIO360_LIB=tools/probe/libvio360_poll.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "global or config5" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_poll.log 2>&1
rc=$?; echo "pytest poll rc=$rc"; tail -3 gpurun_out/pytest_poll.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python3 tools/gba_time.py 10 3 > gpurun_out/gba_base.log 2>&1 || exit 1; echo base; tail -1 gpurun_out/gba_base.log
VIO360_LIB=tools/probe/libvio360_poll.so timeout -k 10 200 python3 tools/gba_time.py 10 3 > gpurun_out/gba_poll.log 2>&1 || exit 1; echo poll; tail -1 gpurun_out/gba_poll.log
rm -rf gpurun_out/pollprof
VIO360_LIB=tools/probe/libvio360_poll.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pollprof -o gba --output-format csv -- python3 tools/gba_time.py 3 1 > gpurun_out/poll_prof.log 2>&1 || exit 1
grep -h trsv gpurun_out/pollprof/*/*kernel_stats.csv | cut -d, -f1-4
