#!/bin/bash
# HBM traffic of one config-2 window solve (10 KF x 200 landmarks, 10 fixed LM iterations, default route
# for one window): one rocprofv3 PMC pass per counter over tools/ba_batch_run.py (BA_CFG=2, W=1, S=3).
# Summary: tools/pmc_summary.py -> gpurun_out/pmc_cfg2/traffic.json (bench.py reads the committed copy,
# profiles/r*_pmc_traffic_cfg2.json, for config2.roofline.traffic).
set -u
mkdir -p gpurun_out/pmc_cfg2
export TMPDIR=/tmp
export BA_CFG=2
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_cfg2/$ctr
  timeout -k 10 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_cfg2/$ctr -o run --output-format csv -- \
      python3 tools/ba_batch_run.py 1 3 > gpurun_out/pmc_cfg2/$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc"; tail -1 gpurun_out/pmc_cfg2/$ctr.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_cfg2 gpurun_out/pmc_cfg2/traffic.json
