#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python tools/ph_solve_stamps.py 1 > gpurun_out/stamps.log 2>&1 || exit 1
timeout -k 10 60 python tools/ph_solve_stamps.py 256 >> gpurun_out/stamps.log 2>&1 || exit 1
cat gpurun_out/stamps.log | grep W=
export VIO_BA_PHASES=1
for w in 1 32; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ph$w -o ph --output-format csv -- python3 tools/ba_batch_run.py $w 10 > gpurun_out/prof_ph$w.log 2>&1 || exit 1
done

unset VIO_BA_PHASES
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "packed or trace" > gpurun_out/pytest_pack.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_pack.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-klt --no-global --no-imu --no-tri --no-resize > gpurun_out/bench_quick.log 2>&1; echo "bench rc=$?"; tail -c 1500 gpurun_out/bench_quick.log
