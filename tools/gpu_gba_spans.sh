#!/bin/bash
# global BA: GPU parity tests, then the device span of the Cholesky + solves per LM iteration (kernel
# trace of tools/gba_time.py 3 1) for each lib[:ENV=VAL]
set -u
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "global or config5" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; }
i=0
for spec in "$@"; do
  i=$((i+1)); lib=${spec%%:*}; env=""; [ "$spec" != "$lib" ] && env=${spec#*:}
  d=gpurun_out/span_${tag}_$i; rm -rf $d
  env $env VIO360_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/gba_time.py 3 1 > $d.log 2>&1 || exit 1
  echo "$(basename $lib) $env $(python3 tools/gba_chol_span.py $(find $d -name '*kernel_trace.csv' | head -1))"
done
