#!/bin/bash
set -u
bash tools/gpu_lanes.sh lanes1 || exit $?
bash tools/gpu_trk7.sh trk8
