#!/bin/bash
# BA parity tests, then the quick timings under both routes: default routing and every non-PnP
# window on the phase kernels (VIO_BA_PHASES=1), plus a kernel trace of the forced-phase run.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ba.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ba_quick.py > gpurun_out/ba_quick.log 2>&1
rc=$?; echo "ba_quick rc=$rc"; grep windows= gpurun_out/ba_quick.log
if [ $rc -ne 0 ]; then exit $rc; fi
VIO_BA_PHASES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ph -o ph --output-format csv -- python3 tools/ba_quick.py > gpurun_out/ba_quick_phases.log 2>&1
rc=$?; echo "ba_quick (phase route) rc=$rc"; grep windows= gpurun_out/ba_quick_phases.log
exit $rc
