#!/bin/bash
# SQ / TCC counters of the config-5 Cholesky kernels (tools/gba_time.py 1 1), one pass per counter group
set -u
mkdir -p gpurun_out/pmc_syrk
export TMPDIR=/tmp
p=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY" "TCC_HIT_sum TCC_MISS_sum"; do
  p=$((p+1)); rm -rf gpurun_out/pmc_syrk/p$p
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_syrk/p$p -o run --output-format csv -- python3 tools/gba_time.py 1 1 > gpurun_out/pmc_syrk/p$p.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(lambda: defaultdict(int))
for f in glob.glob("gpurun_out/pmc_syrk/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("vio360::", "")
        if "chol_" not in n: continue
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[n][r["Counter_Name"]] += 1
for n in acc:
    print(n, {k: round(v / max(1, cnt[n][k])) for k, v in sorted(acc[n].items())})
PY
