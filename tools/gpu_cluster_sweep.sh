set -u
for W in 8 16 32; do
  for R in cluster phases; do
    if [ $R = phases ]; then export VIO_BA_PHASES=1; unset VIO_BA_ROUTE; else export VIO_BA_ROUTE=cluster; unset VIO_BA_PHASES; fi
    timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 > gpurun_out/clsweep_${R}_$W.log 2>&1 || { echo fail $R $W; tail -3 gpurun_out/clsweep_${R}_$W.log; exit 1; }
    echo "$R $(tail -1 gpurun_out/clsweep_${R}_$W.log)"
  done
done
