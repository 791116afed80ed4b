#!/bin/bash
# round-2 refresh: GPU suite, BA timings, bench + kernel stats, PMC traffic (bench workload and the BA step)
set -u
bash tools/gpu_check.sh || exit $?
bash tools/gpu_pmc.sh || exit $?
bash tools/gpu_pmc_ba.sh || exit $?
