#!/bin/bash
# tracker: pipeline timeline (tools/gpu_trk_timeline.sh), then the HBM traffic of the
# config-1 pipeline (FETCH_SIZE / WRITE_SIZE in separate passes over tools/trk_time.py)
set -u
tag=${1:-trk}
bash tools/gpu_trk_timeline.sh $tag || exit $?
mkdir -p gpurun_out/pmc_$tag
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$tag/$ctr
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc_$tag/$ctr -o run --output-format csv -- \
      python3 tools/trk_time.py 10 > gpurun_out/pmc_$tag/$ctr.log 2>&1
  rc=$?; echo "$ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmc_$tag/$ctr.log; exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_$tag gpurun_out/pmc_$tag/traffic.json && python3 - gpurun_out/pmc_$tag/traffic.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
tot = 0.0
for k, v in sorted(d.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches"]):
    if "vio360" in k or any(s in k for s in ("pyr", "gftt", "lk_", "ransac", "disc")):
        print(f"  {k[:48]:48s} n={v['dispatches']:4d} R={v['read_bytes_per_launch']/1e6:7.2f} MB W={v['write_bytes_per_launch']/1e6:6.2f} MB")
PY
