# Round 4: the product's allocation rule for the CG
# pass's streamed buffers (>= 2 GiB each, stream_alloc_bytes) against
# allocations of their own size (SM_TEST_OPTS=pad_alloc=0): interleaved
# bench.py pairs, then per layout the pass's kernel time (rocprofv3 stats) and
# fabric-side counters (read requests, requests in flight, DRAM credit
# stalls). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2 3; do
  SM_TEST_OPTS=pad_alloc=0 timeout -k 10 200 $B > gpurun_out/pad_off_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/pad_on_${i}_$T.log 2>&1 || exit 1
done
P="python3 bench.py --steps 40 --warmup 5 --applies 2 --no-cpu-baseline --no-weak"
for v in off on; do
  if [ $v = off ]; then export SM_TEST_OPTS=pad_alloc=0; else unset SM_TEST_OPTS; fi
  rm -rf gpurun_out/padprof_s_${v}_$T gpurun_out/padprof_c_${v}_$T
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/padprof_s_${v}_$T -o run -- $P > gpurun_out/padprof_s_${v}_$T.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/padprof_c_${v}_$T -o run -- $P > gpurun_out/padprof_c_${v}_$T.log 2>&1 || exit 1
done
