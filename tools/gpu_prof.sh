#!/bin/bash
# The round's profile set of one build, in one gpurun call (each rocprofv3 run is one pass under its own time
# limit; the first failure ends the script).  Sections (SECTIONS env, default all):
#   ks   isolated kernel statistics (--kernel-trace --stats) of the window BA at 1 / 32 / 256 windows
#        (tools/ba_batch_run.py, default route) -> <out>/ks_<W>/
#   pmc  HBM traffic of the 256-window step (FETCH_SIZE / WRITE_SIZE passes) -> <out>/pmc_ba/traffic.json
#   cfg2 HBM traffic of one config-2 window solve -> <out>/pmc_cfg2/traffic.json
#   mix  SQ instruction-mix / MFMA passes: cluster kernel at 1 window, phase kernels at 256, two config-5
#        iterations -> <out>/mix/mix.json
#   gba  config-5 kernel statistics of a 3-iteration solve and per-iteration traffic (3 - 1 iterations) / 2
#   trk  config-1 tracker timeline and traffic
# Usage: SECTIONS="ks pmc" tools/gpu_prof.sh <tag>
set -u
tag=${1:-r6}
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
SECTIONS=${SECTIONS:-"ks pmc cfg2 mix gba trk"}
has() { [[ " $SECTIONS " == *" $1 "* ]]; }
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(tail -1 $out/$name.log | cut -c1-180)"
  return $rc
}
if has ks; then
  for W in 1 32 256; do
    step ks_$W 240 rocprofv3 --kernel-trace --stats -d $out/ks_$W -o run --output-format csv -- python3 tools/ba_batch_run.py $W 10 || exit 1
  done
fi
if has pmc; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step pmc_ba_$ctr 240 rocprofv3 --pmc $ctr -d $out/pmc_ba/$ctr -o run --output-format csv -- python3 tools/ba_batch_run.py 256 3 || exit 1
  done
  python3 tools/pmc_summary.py $out/pmc_ba $out/pmc_ba/traffic.json || exit 1
fi
if has cfg2; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    BA_CFG=2 step pmc_cfg2_$ctr 120 rocprofv3 --pmc $ctr -d $out/pmc_cfg2/$ctr -o run --output-format csv -- python3 tools/ba_batch_run.py 1 3 || exit 1
  done
  python3 tools/pmc_summary.py $out/pmc_cfg2 $out/pmc_cfg2/traffic.json || exit 1
fi
if has mix; then
  P1="SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_MFMA_MOPS_F64,SQ_INSTS_VMEM,SQ_INSTS_LDS"
  P2="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_SALU,SQ_WAIT_ANY,SQ_INSTS_VALU_MFMA_F64,GRBM_GUI_ACTIVE"
  step mix_cl1_p1 240 rocprofv3 --pmc $P1 -d $out/mix/cl1_p1 -o run --output-format csv -- python3 tools/ba_batch_run.py 1 10 || exit 1
  step mix_cl1_p2 240 rocprofv3 --pmc $P2 -d $out/mix/cl1_p2 -o run --output-format csv -- python3 tools/ba_batch_run.py 1 10 || exit 1
  VIO_BA_PHASES=1 step mix_ph256_p1 240 rocprofv3 --pmc $P1 -d $out/mix/ph256_p1 -o run --output-format csv -- python3 tools/ba_batch_run.py 256 3 || exit 1
  VIO_BA_PHASES=1 step mix_ph256_p2 240 rocprofv3 --pmc $P2 -d $out/mix/ph256_p2 -o run --output-format csv -- python3 tools/ba_batch_run.py 256 3 || exit 1
  step mix_gba_p1 300 rocprofv3 --pmc $P1 -d $out/mix/gba_p1 -o run --output-format csv -- python3 tools/gba_run.py 2 || exit 1
  step mix_gba_p2 300 rocprofv3 --pmc $P2 -d $out/mix/gba_p2 -o run --output-format csv -- python3 tools/gba_run.py 2 || exit 1
  python3 tools/pmc_mix_summary.py $out/mix $out/mix/mix.json || exit 1
fi
if has gba; then
  step gba_ks 300 rocprofv3 --kernel-trace --stats -d $out/gba_ks -o run --output-format csv -- python3 tools/gba_run.py 3 || exit 1
  for n in 1 3; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      mkdir -p $out/pmc_gba/n$n
      step pmc_gba_n${n}_$ctr 240 rocprofv3 --pmc $ctr -d $out/pmc_gba/n$n/$ctr -o run --output-format csv -- python3 tools/gba_run.py $n || exit 1
    done
  done
  python3 tools/pmc_gba_summary.py $out/pmc_gba $out/pmc_gba/traffic_gba.json || exit 1
fi
if has trk; then
  step trk_trace 300 rocprofv3 --kernel-trace -d $out/trk_trace -o run --output-format csv -- python3 tools/trk_time.py 20 || exit 1
  f=$(find $out/trk_trace -name "*kernel_trace.csv" | head -1)
  python3 tools/trk_timeline.py $f > $out/trk_timeline.log && tail -25 $out/trk_timeline.log
  rm -rf $out/trk_trace
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step pmc_trk_$ctr 120 rocprofv3 --pmc $ctr -d $out/pmc_trk/$ctr -o run --output-format csv -- python3 tools/trk_time.py 10 || exit 1
  done
  python3 tools/pmc_summary.py $out/pmc_trk $out/pmc_trk/traffic.json || exit 1
fi
echo done
