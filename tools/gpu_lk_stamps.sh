export TMPDIR=/tmp; mkdir -p gpurun_out
VIO360_LIB=tools/probe/libvio360_dbg.so timeout -k 10 120 python3 tools/trk_time.py 1 > gpurun_out/r6e_lk_stamps.log 2>&1 || { tail -20 gpurun_out/r6e_lk_stamps.log; exit 1; }
grep -E "^lk pt" gpurun_out/r6e_lk_stamps.log | tail -14
