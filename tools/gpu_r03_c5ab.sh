# Config 5 (8192^2, one GPU) time to solution under three field layouts:
# one pool (tools/ab/libsm_hip_pool.so), own allocations of >= 2 GiB (the
# product), own allocations of >= 4x the field (tools/ab/libsm_hip_x4.so). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for i in 1 2; do
  SM_LIB_PATH=tools/ab/libsm_hip_pool.so timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > gpurun_out/c5_pool_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > gpurun_out/c5_cur_${i}_$T.log 2>&1 || exit 1
  SM_LIB_PATH=tools/ab/libsm_hip_x4.so timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > gpurun_out/c5_x4_${i}_$T.log 2>&1 || exit 1
done
