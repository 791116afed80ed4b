#!/bin/bash
# global BA triangular-solve variants (tools/probe/libvio360_<v>.so) vs the in-tree library:
# parity tests, per-iteration time, kernel stats
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/gba_time.py 10 3 > gpurun_out/gba_base.log 2>&1 || exit 1; echo base; tail -1 gpurun_out/gba_base.log
for v in "$@"; do
  VIO360_LIB=tools/probe/libvio360_$v.so timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "global or config5" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -2 gpurun_out/pytest_$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  VIO360_LIB=tools/probe/libvio360_$v.so timeout -k 10 200 python3 tools/gba_time.py 10 3 > gpurun_out/gba_$v.log 2>&1 || exit 1; echo $v; tail -1 gpurun_out/gba_$v.log
  rm -rf gpurun_out/prof_$v
  VIO360_LIB=tools/probe/libvio360_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o gba --output-format csv -- python3 tools/gba_time.py 3 1 > gpurun_out/prof_$v.log 2>&1 || exit 1
done
