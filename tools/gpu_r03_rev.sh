# Round 3: odd CG passes marching backwards over reversed tiles (rev) against
# forward marches (SM_TEST_OPTS=rev=0), interleaved A/B/A/B bench runs, then the
# CG parity subset. Tag $1. Outputs under gpurun_out/.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/rev_on${i}_$T.log 2>&1 || exit 1
  SM_TEST_OPTS=rev=0 timeout -k 10 200 $B > gpurun_out/rev_off${i}_$T.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cg_paths_gpu.py tests/test_gpu_large.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/rev_tests_$T.log 2>&1
