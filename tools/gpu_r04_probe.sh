# Round 4: the placement probe at context creation (place_probe, default 3
# candidate sets) -- the CG parity subset with it on, then interleaved
# bench.py pairs against no probe (SM_TEST_OPTS=place_probe=1). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_cg_paths_gpu.py tests/test_gpu_large.py tests/test_rccl_loopback_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/probe_tests_$T.log 2>&1 || exit 1
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2 3 4; do
  SM_TEST_OPTS=place_probe=1 timeout -k 10 200 $B > gpurun_out/probe_off_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/probe_on_${i}_$T.log 2>&1 || exit 1
done
