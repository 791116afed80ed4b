#!/bin/bash
# ph_back chunk-0 breakdown (diagnostic build tools/probe/libvio360_bst.so: slots 6/15/7/13/14 = loads+jac,
# landmark back-substitution, candidate eval + Jacobian, landmark sums, pose partials)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 1 256; do VIO360_LIB=tools/probe/libvio360_bst.so timeout -k 10 120 python3 tools/ph_solve_stamps.py $w > gpurun_out/bst$w.log 2>&1 || exit 1; grep schur gpurun_out/bst$w.log; done
