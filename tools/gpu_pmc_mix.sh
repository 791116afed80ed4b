#!/bin/bash
# Instruction mix / MFMA utilisation of the BA kernels: rocprofv3 PMC passes (<= 8 SQ counters each,
# no tracing domains) over (a) the 256-window config-4 shard on the single-kernel route, (b) the same
# on the phase route, (c) two LM iterations of config-5 global BA.  Summary: tools/pmc_mix_summary.py.
set -u
mkdir -p gpurun_out/pmcmix
export TMPDIR=/tmp
P1="SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_MFMA_MOPS_F64,SQ_INSTS_VMEM,SQ_INSTS_LDS"
P2="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_SALU,SQ_WAIT_ANY,SQ_INSTS_VALU_MFMA_F64"
run() {  # name env counters cmd...
  local name=$1 envs=$2 ctrs=$3; shift 3
  rm -rf gpurun_out/pmcmix/$name
  env $envs timeout -k 10 240 rocprofv3 --pmc $ctrs -d gpurun_out/pmcmix/$name -o run --output-format csv -- "$@" \
      > gpurun_out/pmcmix/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/pmcmix/$name.log | cut -c1-200
  return $rc
}
run mono_p1 VIO_BA_MONOLITHIC=1 $P1 python3 tools/ba_batch_run.py 256 3 &&
run mono_p2 VIO_BA_MONOLITHIC=1 $P2 python3 tools/ba_batch_run.py 256 3 &&
run ph_p1 VIO_BA_PHASES=1 $P1 python3 tools/ba_batch_run.py 256 3 &&
run ph_p2 VIO_BA_PHASES=1 $P2 python3 tools/ba_batch_run.py 256 3 &&
run gba_p1 X=1 $P1 python3 tools/gba_run.py 2 &&
run gba_p2 X=1 $P2 python3 tools/gba_run.py 2 &&
python3 tools/pmc_mix_summary.py gpurun_out/pmcmix gpurun_out/pmcmix/mix.json
