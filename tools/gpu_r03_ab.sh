# Interleaved A/B of the product build against tools/ab/libsm_hip_base.so
# (SM_LIB_PATH) on bench.py (200 steps), FETCH/WRITE counters of the new
# build's CG pass, then the CG parity subset. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2 3; do
  SM_LIB_PATH=tools/ab/libsm_hip_base.so timeout -k 10 200 $B > gpurun_out/ab_base_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/ab_new_${i}_$T.log 2>&1 || exit 1
done
P="python3 bench.py --steps 10 --warmup 2 --applies 2 --no-cpu-baseline --no-weak"
rm -rf gpurun_out/abpmc_f_$T gpurun_out/abpmc_w_$T
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/abpmc_f_$T -o run -- $P > gpurun_out/abpmc_f_$T.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/abpmc_w_$T -o run -- $P > gpurun_out/abpmc_w_$T.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cg_paths_gpu.py tests/test_gpu_large.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab_tests_$T.log 2>&1
