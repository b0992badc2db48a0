# Round 3: recompute-Ad pass march schedules, interleaved bench runs
# (rev=1: odd passes backwards, the default; rev=2: x-adjacent chunks in
# opposite directions as well; rev=0: all forward), FETCH/WRITE counters of
# the pass for rev 1 and 2, then the CG parity subset under rev=2. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2; do
  for r in 2 1; do
    SM_TEST_OPTS=rev=$r timeout -k 10 200 $B > gpurun_out/alt_r${r}_${i}_$T.log 2>&1 || exit 1
  done
done
P="python3 bench.py --steps 10 --warmup 2 --applies 2 --no-cpu-baseline --no-weak"
for r in 2; do
  rm -rf gpurun_out/altpmc_f$r_$T gpurun_out/altpmc_w$r_$T
  SM_TEST_OPTS=rev=$r timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/altpmc_f${r}_$T -o run -- $P > gpurun_out/altpmc_f${r}_$T.log 2>&1 || exit 1
  SM_TEST_OPTS=rev=$r timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/altpmc_w${r}_$T -o run -- $P > gpurun_out/altpmc_w${r}_$T.log 2>&1 || exit 1
done
SM_TEST_OPTS=rev=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cg_paths_gpu.py tests/test_gpu_large.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/alt_tests_$T.log 2>&1
