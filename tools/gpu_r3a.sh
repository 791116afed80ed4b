#!/bin/bash
# round-3 check: GPU parity suite, default bench line, isolated per-workload kernel stats
set -u
mkdir -p gpurun_out
tag=${1:-r3a}
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/pytest_$tag.log | head -5; exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$tag.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$tag.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_prof_ba.sh $tag
