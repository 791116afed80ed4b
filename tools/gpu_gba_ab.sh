#!/bin/bash
# global BA: GPU parity tests, then per-LM-iteration time of config 5 per library (tools/gba_time.py),
# 3 rounds.  args: tag lib[:ENV=VAL] ...
set -u
mkdir -p gpurun_out
tag=${1:-gba}; shift
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "global or config5" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; }
for rep in 1 2 3; do
  for spec in "$@"; do
    lib=${spec%%:*}; env=""; [ "$spec" != "$lib" ] && env=${spec#*:}
    echo "$(basename $lib) $env $(env $env VIO360_LIB=$lib timeout -k 10 200 python3 tools/gba_time.py 5 3 2>&1 | grep -v amdgpu.ids | tail -1)" || exit 1
  done
done
