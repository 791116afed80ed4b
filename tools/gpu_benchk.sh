#!/bin/bash
# full default bench (CPU baselines included), tracker leg summary
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
python3 -c "
import json
l=[x for x in open('gpurun_out/bench.log') if x.startswith('{')][-1]
d=json.loads(l); print('value', d['value'], 'klt', d['erp_klt']['device_ms_per_step'], d['erp_klt']['stage_ms'], 'gba', d['global_ba']['ms_per_iteration'])
"
