set -u
export TMPDIR=/tmp
for W in 16 32 64 128; do
  for v in 8 256; do
    echo "IMU_BACK_MAX=$v $(VIO_BA_IMU_BACK_MAX=$v timeout -k 10 120 python3 tools/ba_batch_run.py $W 30 2>&1 | grep -v amdgpu.ids | tail -1)" || exit 1
  done
done
