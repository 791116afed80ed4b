set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probe/cholmw_probe > gpurun_out/cholmw_h.log 2>&1; cat gpurun_out/cholmw_h.log
timeout -k 10 60 ./tools/probe/lat_probe > gpurun_out/lat_h.log 2>&1; cat gpurun_out/lat_h.log
