#!/bin/bash
# tracker parity + stage times + kernel trace; global BA parity + per-iteration time
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_trk4.sh || exit $?
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "global or config5" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gba.log 2>&1
rc=$?; echo "pytest gba rc=$rc"; tail -3 gpurun_out/pytest_gba.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python3 tools/gba_time.py 5 > gpurun_out/gba_time.log 2>&1 || exit 1
grep gba gpurun_out/gba_time.log
for m in 0 24 96; do VIO_GBA_FUSE_M=$m timeout -k 10 200 python3 tools/gba_time.py 5 >> gpurun_out/gba_time.log 2>&1 || exit 1; echo "fuse_m=$m"; tail -1 gpurun_out/gba_time.log; done
