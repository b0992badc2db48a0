# Round 4: placement probe with 1 (none), 5 and 8 (the default) candidate
# sets, interleaved bench.py runs, + the probe test. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cg_paths_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread -k "placement" > gpurun_out/probe2_tests_$T.log 2>&1 || exit 1
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2 3; do
  for k in 1 5 8; do
    SM_TEST_OPTS=place_probe=$k timeout -k 10 200 $B > gpurun_out/probe2_k${k}_${i}_$T.log 2>&1 || exit 1
  done
done
