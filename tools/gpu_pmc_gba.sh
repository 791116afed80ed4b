#!/bin/bash
# HBM traffic of one config-5 LM iteration (global BA): FETCH_SIZE / WRITE_SIZE, one rocprofv3 PMC pass
# per counter, over 1- and 3-iteration solves (tools/gba_run.py); the per-iteration bytes are the
# difference / 2 (set-up, first linearisation and the chi2 pass cancel).  Summary: tools/pmc_gba_summary.py
set -u
mkdir -p gpurun_out/pmc_gba
export TMPDIR=/tmp
for n in 1 3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_gba/n$n/$ctr
    rm -rf $d
    mkdir -p gpurun_out/pmc_gba/n$n
    timeout -k 10 240 rocprofv3 --pmc $ctr -d $d -o run --output-format csv -- python3 tools/gba_run.py $n > $d.log 2>&1
    rc=$?; echo "n=$n $ctr rc=$rc $(tail -1 $d.log | cut -c1-160)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
python3 tools/pmc_gba_summary.py gpurun_out/pmc_gba gpurun_out/pmc_gba/traffic_gba.json
