#!/bin/bash
# round-3 iteration: GPU parity suite, quick BA timings (1 / 256 windows), ph_solve stamp breakdown
set -u
mkdir -p gpurun_out
tag=${1:-r3}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log; grep -E "^FAILED|Error" gpurun_out/pytest_$tag.log | head -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/ba_quick.py > gpurun_out/ba_quick_$tag.log 2>&1
rc2=$?; echo "ba_quick rc=$rc2"; grep -E "windows=|parity|cfg|pnp|local" gpurun_out/ba_quick_$tag.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
for W in 1 32 256; do timeout -k 10 120 python -u tools/ph_solve_stamps.py $W > gpurun_out/stamps_${tag}_$W.log 2>&1 || exit $?; done
grep -E "chol|solve|prep|schur" gpurun_out/stamps_${tag}_1.log
bash tools/gpu_prof_ba.sh $tag || exit $?
exit $rc
