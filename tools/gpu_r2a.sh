#!/bin/bash
# round-2 check: GPU suite, trace dumps of both BA routes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/trace_dump.py phases > gpurun_out/trace_phases.log 2>&1
rc=$?; echo "trace phases rc=$rc"; cat gpurun_out/trace_phases.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/trace_dump.py mono > gpurun_out/trace_mono.log 2>&1
rc=$?; echo "trace mono rc=$rc"; cat gpurun_out/trace_mono.log | tail -5
exit $rc
