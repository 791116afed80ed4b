#!/bin/bash
# reduced-solve probes (tools/probe/cholmw_probe) and the pivot-chain latency constants (lat_probe)
set -u
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probe/cholmw_probe > gpurun_out/cholmw_i.log 2>&1; cat gpurun_out/cholmw_i.log
timeout -k 10 60 ./tools/probe/lat_probe > gpurun_out/lat_i.log 2>&1; cat gpurun_out/lat_i.log
