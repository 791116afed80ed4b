#!/bin/bash
# full GPU suite, smoke(), default bench line
set -u
mkdir -p gpurun_out
tag=${1:-r3c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -5 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_$tag.log
exit $rc
