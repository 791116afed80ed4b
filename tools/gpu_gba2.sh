#!/bin/bash
# global BA parity + per-iteration time at several fused-step thresholds
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "global or config5" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gba.log 2>&1
rc=$?; echo "pytest gba rc=$rc"; tail -3 gpurun_out/pytest_gba.log
if [ $rc -ne 0 ]; then exit $rc; fi
rm -f gpurun_out/gba_time.log
for m in 32 48 64 96; do VIO_GBA_FUSE_M=$m timeout -k 10 200 python3 tools/gba_time.py 10 >> gpurun_out/gba_time.log 2>&1 || exit 1; echo "fuse_m=$m"; tail -1 gpurun_out/gba_time.log; done
