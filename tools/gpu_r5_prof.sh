#!/bin/bash
# Round-5 profile set of the shipped build (one gpurun call):
#  (1) isolated kernel statistics (rocprofv3 --kernel-trace --stats) of the window BA at 1 / 32 / 256
#      windows on the default route (tools/ba_batch_run.py);
#  (2) HBM traffic of the 256-window step (FETCH_SIZE / WRITE_SIZE passes; tools/pmc_summary.py here);
#  (3) SQ instruction-mix / MFMA passes of this round's kernels: the cluster route at 1 window
#      (ph_cluster_kernel), the phase route at 256 windows (ph_schur / ph_back / ph_solve / ph_prep),
#      two config-5 LM iterations (chol_chain_kernel / chol_syrk_kernel / gba_schur_kernel).
# Each rocprofv3 run is one pass under its own time limit; the first failure ends the script.
set -u
tag=${1:-r5a}
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(tail -1 $out/$name.log | cut -c1-180)"
  return $rc
}
for W in 1 32 256; do
  step ks_$W 240 rocprofv3 --kernel-trace --stats -d $out/ks_$W -o run --output-format csv -- python3 tools/ba_batch_run.py $W 10 || exit 1
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  step pmc_ba_$ctr 240 rocprofv3 --pmc $ctr -d $out/pmc_ba/$ctr -o run --output-format csv -- python3 tools/ba_batch_run.py 256 3 || exit 1
done
P1="SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_MFMA_MOPS_F64,SQ_INSTS_VMEM,SQ_INSTS_LDS"
P2="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_SALU,SQ_WAIT_ANY,SQ_INSTS_VALU_MFMA_F64,GRBM_GUI_ACTIVE"
step mix_cl1_p1 240 rocprofv3 --pmc $P1 -d $out/mix/cl1_p1 -o run --output-format csv -- python3 tools/ba_batch_run.py 1 10 || exit 1
step mix_cl1_p2 240 rocprofv3 --pmc $P2 -d $out/mix/cl1_p2 -o run --output-format csv -- python3 tools/ba_batch_run.py 1 10 || exit 1
export VIO_BA_PHASES=1
step mix_ph256_p1 240 rocprofv3 --pmc $P1 -d $out/mix/ph256_p1 -o run --output-format csv -- python3 tools/ba_batch_run.py 256 3 || exit 1
step mix_ph256_p2 240 rocprofv3 --pmc $P2 -d $out/mix/ph256_p2 -o run --output-format csv -- python3 tools/ba_batch_run.py 256 3 || exit 1
unset VIO_BA_PHASES
step mix_gba_p1 300 rocprofv3 --pmc $P1 -d $out/mix/gba_p1 -o run --output-format csv -- python3 tools/gba_run.py 2 || exit 1
step mix_gba_p2 300 rocprofv3 --pmc $P2 -d $out/mix/gba_p2 -o run --output-format csv -- python3 tools/gba_run.py 2 || exit 1
echo done
