# round 5: CG pass tile order t-block-major within each XCD (ra_remap=2) against
# the default (1): L2 / fabric counters + interleaved timing; parity subset on 2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r05i_*
P="python3 bench.py --steps 10 --warmup 2 --applies 4 --no-cpu-baseline --no-weak --evolved-trajectories 0"
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak --evolved-trajectories 0"
for v in ra_remap=2 ra_remap=1; do
  export SM_TEST_OPTS=$v
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/r05i_pmc_$v -o run -- $P > gpurun_out/r05i_pmc_$v.log 2>&1 || exit 1
done
for r in 1 2; do for v in ra_remap=2 ra_remap=1; do
  export SM_TEST_OPTS=$v
  timeout -k 10 200 $B > gpurun_out/r05i_bench${r}_$v.log 2>&1 || exit 1
done; done
export SM_TEST_OPTS=ra_remap=2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_large.py -k "l4096 and cg" > gpurun_out/r05i_parity.log 2>&1
