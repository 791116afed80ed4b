#!/bin/bash
# tracker GPU tests, then the pipeline timeline and same-box A/B (tools/gpu_ab_trk.sh) against ab/*.so
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tracker_gpu.py tests/test_frontend_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_trk.log 2>&1 || { tail -30 gpurun_out/pytest_trk.log; exit 1; }
tail -2 gpurun_out/pytest_trk.log
bash tools/gpu_trk_timeline.sh ${TAG:-ab} || exit 1
bash tools/gpu_ab_trk.sh 360_visual_inertial_odometry_amd/libvio360.so "$@"
