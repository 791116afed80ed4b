#!/bin/bash
# Diagnostic tracker build: tracker.hip with the RANSAC stamps (TRK_STAMPS) and the GFTT selection breakdown
# (GFTT_DEBUG), linked with the other objects of the in-tree build into tools/probe/libvio360_dbg.so
# (use: VIO360_LIB=tools/probe/libvio360_dbg.so python3 tools/trk_time.py 5).  Built here, on the CPU.
set -e
root=$(cd "$(dirname "$0")/../.." && pwd)
cd "$root/360_visual_inertial_odometry_amd/csrc"
make -s
mkdir -p /tmp/trkdbg
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -ffp-contract=off \
  -DTRK_STAMPS -DGFTT_DEBUG -w -c tracker.hip -o /tmp/trkdbg/tracker.o
objs=$(ls build/*.o | grep -v '^build/tracker\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$root/tools/probe/libvio360_dbg.so" $objs /tmp/trkdbg/tracker.o
echo "built $root/tools/probe/libvio360_dbg.so"
