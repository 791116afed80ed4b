#!/bin/bash
set -u
bash tools/gpu_gs2.sh gs2 || exit $?
bash tools/gpu_trk7.sh trk11
