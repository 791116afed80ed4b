#!/bin/bash
# global BA (config 5) A/B of the Schur assembly: per-iteration time with the lane-per-block kernel and
# with the former wave-per-block kernel (VIO_GBA_SCHUR=wave), kernel statistics of 2 iterations, then
# the global-BA GPU tests
set -u
tag=${1:-x}
out=gpurun_out/qgba_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/gba_time.py 8 3 > $out/t_lane.log 2>&1 || { tail -5 $out/t_lane.log; exit 1; }
tail -1 $out/t_lane.log
VIO_GBA_SCHUR=r4 timeout -k 10 200 python3 tools/gba_time.py 8 3 > $out/t_wave.log 2>&1 || { tail -5 $out/t_wave.log; exit 1; }
echo "r4: $(tail -1 $out/t_wave.log)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/ks -o run --output-format csv -- python3 tools/gba_run.py 2 > $out/ks.log 2>&1 || { tail -5 $out/ks.log; exit 1; }
VIO_GBA_SCHUR=r4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/ks_r4 -o run --output-format csv -- python3 tools/gba_run.py 2 > $out/ks_r4.log 2>&1 || { tail -5 $out/ks_r4.log; exit 1; }
grep gba_schur $out/ks_r4/run_kernel_stats.csv | cut -c1-120
head -6 $out/ks/run_kernel_stats.csv | cut -c1-150
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "global or config5" > $out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log; exit $rc
fi
