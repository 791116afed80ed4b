#!/bin/bash
# I-cache / issue-stall counters of the BA window kernel and the tracker kernels (one PMC pass each).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST_ANY\|SQ_WAVE_CYCLES\|SQ_INSTS_VALU\b\|SQ_ACTIVE_INST_ANY" gpurun_out/pmc/avail.txt | sort -u | head -20
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY -d gpurun_out/pmc/ic -o ic --output-format csv -- python3 bench.py --steps 2 --warmup 1 --windows 256 --no-cpu-baseline --no-global --klt-steps 3 > gpurun_out/pmc/ic.log 2>&1
echo "rc=$?"
