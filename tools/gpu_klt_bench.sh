#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/trk_time.py 20 > gpurun_out/trk_a.log 2>&1 || exit 1; grep total gpurun_out/trk_a.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-global > gpurun_out/bench_k.log 2>&1 || exit 1
python3 -c "
import json
l=[x for x in open('gpurun_out/bench_k.log') if x.startswith('{')][-1]
d=json.loads(l); print('bench klt', d['erp_klt']['device_ms_per_step'], d['erp_klt']['stage_ms'])
"
