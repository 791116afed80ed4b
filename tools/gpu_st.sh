#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/ph_solve_stamps.py 256 >> gpurun_out/stamps.log 2>&1 || exit 1
grep -E "schur" gpurun_out/stamps.log
