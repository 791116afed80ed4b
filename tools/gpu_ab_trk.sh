#!/bin/bash
# A/B of libvio360 builds / settings on one box: config-1 tracker pipeline time (tools/trk_time.py), 3 rounds.
# args: lib[:ENV=VAL] ...
set -u
for rep in 1 2 3; do
  for spec in "$@"; do
    lib=${spec%%:*}; env=""; [ "$spec" != "$lib" ] && env=${spec#*:}
    echo "$(basename $lib) $env $(env $env VIO360_LIB=$lib timeout -k 10 120 python3 tools/trk_time.py 50 2>&1 | grep -E 'total_ms|stage_ms' | tr '\n' ' ')" || exit 1
  done
done
