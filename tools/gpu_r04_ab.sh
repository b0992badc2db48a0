# Round 4: interleaved bench.py A/B/C of up to three CG-pass variants
#   base: tools/ab/libsm_hip_base.so (the previous build, SM_LIB_PATH)
#   v1:   this build with SM_TEST_OPTS=$V1_OPTS (default cshift=0)
#   v2:   this build with its defaults
# then FETCH/WRITE counters of v1 and v2's CG pass, and the CG parity subset
# of this build. Tag $1. Summaries: tools/ab_summary.py.
export TMPDIR=/tmp
T=${1:-cur}
V1_OPTS=${V1_OPTS:-cshift=0}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2 3; do
  SM_LIB_PATH=tools/ab/libsm_hip_base.so timeout -k 10 200 $B > gpurun_out/ab_base_${i}_$T.log 2>&1 || exit 1
  SM_TEST_OPTS=$V1_OPTS timeout -k 10 200 $B > gpurun_out/ab_v1_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/ab_new_${i}_$T.log 2>&1 || exit 1
done
P="python3 bench.py --steps 10 --warmup 2 --applies 2 --no-cpu-baseline --no-weak"
for v in v1 new; do
  if [ $v = v1 ]; then export SM_TEST_OPTS=$V1_OPTS; else unset SM_TEST_OPTS; fi
  rm -rf gpurun_out/abpmc_f_${v}_$T gpurun_out/abpmc_w_${v}_$T
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/abpmc_f_${v}_$T -o run -- $P > gpurun_out/abpmc_f_${v}_$T.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/abpmc_w_${v}_$T -o run -- $P > gpurun_out/abpmc_w_${v}_$T.log 2>&1 || exit 1
done
unset SM_TEST_OPTS
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cg_paths_gpu.py tests/test_gpu_large.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab_tests_$T.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -k link_angle -x -v --timeout 120 --timeout-method thread > gpurun_out/ab_dist_tests_$T.log 2>&1
