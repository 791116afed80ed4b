#!/bin/bash
set -u
bash tools/gpu_trk7.sh trk9 || exit $?
bash tools/gpu_measure_r3.sh
