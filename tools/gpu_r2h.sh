#!/bin/bash
# BA parity after a solver change + ph_solve breakdown + BA timings; tracker stage times + GFTT select breakdown
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ba.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps.log 2>&1 || exit 1
grep -E "chol|solve" gpurun_out/stamps.log
timeout -k 10 300 python3 tools/ba_quick.py > gpurun_out/ba_quick.log 2>&1 || exit 1
grep -E "windows=|cfg3" gpurun_out/ba_quick.log
bash tools/gpu_trk3.sh
