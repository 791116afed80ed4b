#!/bin/bash
# round-6 window-BA session: the BA GPU suite on the working tree, then the same-box A/B of the HEAD build
# (tools/probe/libvio360_base.so) against the working tree (tools/probe/libvio360_lb4.so copy) at 1 / 32 / 256 windows
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py > gpurun_out/r6g_ba_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6g_ba_tests.log; exit 1; }
tail -2 gpurun_out/r6g_ba_tests.log
ROUNDS=3 bash tools/ab_ba.sh late tools/probe/libvio360_base.so tools/probe/libvio360_lb4.so > gpurun_out/r6g_ab_back.log 2>&1 || { echo "ab failed"; cat gpurun_out/r6g_ab_back.log; exit 1; }
cat gpurun_out/r6g_ab_back.log
