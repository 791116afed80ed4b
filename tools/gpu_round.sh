#!/bin/bash
# One gpurun call's round check: the full GPU suite, smoke(), the default bench line.  Logs under
# gpurun_out/<tag>/.  Usage: tools/gpu_round.sh <tag>
set -u
tag=${1:-r6}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" $out/pytest_gpu.log | head -8; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 500 python -u bench.py > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $out/bench.log
exit $rc
