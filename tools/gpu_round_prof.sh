#!/bin/bash
# GPU suite + smoke + bench (tools/gpu_round.sh TAG), then the rocprofv3 kernel statistics of a short
# bench run (the summary committed under profiles/ next to the bench line).  usage: tools/gpu_round_prof.sh TAG
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r4}
bash tools/gpu_round.sh $tag || exit 1
rm -rf gpurun_out/prof_bench_$tag
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_$tag -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_bench_$tag.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
