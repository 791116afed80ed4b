#!/bin/bash
# Instruction-cache behaviour of the window-BA kernels: one rocprofv3 PMC pass (SQ/SQC counters only,
# no tracing domains) over one config-3 window (cluster route) and the 256-window shard (phase route).
set -u
mkdir -p gpurun_out/pmcic
export TMPDIR=/tmp
C="SQC_ICACHE_REQ,SQC_ICACHE_HITS,SQC_ICACHE_MISSES,SQC_ICACHE_MISSES_DUPLICATE,SQ_IFETCH,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES"
run() {  # name W
  rm -rf gpurun_out/pmcic/$1
  timeout -k 10 120 rocprofv3 --pmc $C -d gpurun_out/pmcic/$1 -o run --output-format csv -- python3 tools/ba_batch_run.py $2 3 \
      > gpurun_out/pmcic/$1.log 2>&1
  local rc=$?; echo "$1 rc=$rc"; tail -1 gpurun_out/pmcic/$1.log | cut -c1-200
  return $rc
}
run w1 1 && run w256 256
