#!/bin/bash
# Address-translation behaviour of the phase kernels at 256 windows: the ph_prep probe (kernel statistics
# + stamps: which mode this box is in), then one rocprofv3 PMC pass of UTCL1 counters (no tracing domains).
set -u
tag=${1:-x}
bash tools/gpu_prep_probe.sh $tag || exit 1
mkdir -p gpurun_out/tlb_$tag
export TMPDIR=/tmp
C="TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_REQUEST_sum,TCP_UTCL1_SERIALIZATION_STALL_sum,GRBM_GUI_ACTIVE,GRBM_UTCL2_BUSY"
timeout -k 10 120 rocprofv3 --pmc $C -d gpurun_out/tlb_$tag/pmc -o run --output-format csv -- python3 tools/ba_batch_run.py 256 3 \
    > gpurun_out/tlb_$tag/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -3 gpurun_out/tlb_$tag/pmc.log; exit 1; }
python3 tools/pmc_counters.py gpurun_out/tlb_$tag/pmc
