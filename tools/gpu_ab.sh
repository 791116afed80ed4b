#!/bin/bash
# A/B of a BA build variant (tools/probe/libvio360_<v>.so) against the in-tree library: ba_quick timings
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
v=$1
timeout -k 10 200 python3 tools/ba_quick.py > gpurun_out/ba_quick_base.log 2>&1 || exit 1
echo base; grep -E "windows=" gpurun_out/ba_quick_base.log
VIO360_LIB=tools/probe/libvio360_$v.so timeout -k 10 200 python3 tools/ba_quick.py > gpurun_out/ba_quick_$v.log 2>&1 || exit 1
echo $v; grep -E "windows=|cfg3" gpurun_out/ba_quick_$v.log
