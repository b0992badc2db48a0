# round 5: (1) RCCL loopback timeline at 4096x512 (kernel trace, csv) and the
# t-shard apply split A/B; (2) the CG pass's L2 / fabric counters under the
# march schedules and tile orders, with timing pairs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r05h_*
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05h_lbtrace -o run -- python -u tools/loopback_probe.py --shapes 4096x512 --iters 100 --rounds 1 > gpurun_out/r05h_lbtrace.log 2>&1 &&
SM_TEST_OPTS=apply_split=1 timeout -k 10 300 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 3 > gpurun_out/r05h_split1.log 2>&1 &&
SM_TEST_OPTS=apply_split=0 timeout -k 10 300 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 3 > gpurun_out/r05h_split0.log 2>&1 || exit 1
P="python3 bench.py --steps 10 --warmup 2 --applies 4 --no-cpu-baseline --no-weak --evolved-trajectories 0"
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak --evolved-trajectories 0"
for v in default rev=1 rev=0 ra_remap=0; do
  if [ $v = default ]; then unset SM_TEST_OPTS; else export SM_TEST_OPTS=$v; fi
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/r05h_pmc_$v -o run -- $P > gpurun_out/r05h_pmc_$v.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/r05h_bench_$v.log 2>&1 || exit 1
done
unset SM_TEST_OPTS
for v in default rev=1 rev=0 ra_remap=0; do
  if [ $v = default ]; then unset SM_TEST_OPTS; else export SM_TEST_OPTS=$v; fi
  timeout -k 10 200 $B > gpurun_out/r05h_bench2_$v.log 2>&1 || exit 1
done
