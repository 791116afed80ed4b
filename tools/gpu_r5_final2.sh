#!/bin/bash
# Round-5 profile set, part 2 (part 1: tools/gpu_r5_prof.sh): PMC HBM traffic of a config-5 LM iteration
# (tools/gpu_pmc_gba.sh), of the config-1 tracker pipeline with its timeline (tools/gpu_trk_pmc.sh), of a
# config-2 solve (tools/gpu_pmc_cfg2.sh), and the instruction-cache pass (tools/gpu_pmc_icache.sh).
# Each rocprofv3 run is one pass under its own time limit; the first failure ends the script.
set -u
tag=${1:-r5b}
bash tools/gpu_pmc_gba.sh || exit 1
bash tools/gpu_trk_pmc.sh $tag || exit 1
bash tools/gpu_pmc_cfg2.sh || exit 1
bash tools/gpu_pmc_icache.sh || exit 1
echo done
