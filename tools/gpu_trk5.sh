#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 -c "
import torch, ctypes
l=ctypes.CDLL(None)
" >/dev/null 2>&1
timeout -k 10 120 python3 tools/trk_time.py 30 > gpurun_out/trk_time.log 2>&1 || exit 1
cat gpurun_out/trk_time.log
