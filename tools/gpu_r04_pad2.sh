# Round 4: the CG pass under five placements of its
# streamed buffers (SM_TEST_OPTS=pad_alloc=N, sm_ctx.h): 1 >= 2 GiB each (the
# default), 0 own size, 2 >= 1 GiB, 3 own size + hipDeviceMallocContiguous,
# 4 own-size physical memory mapped at a 2 GiB-aligned address (hipMemCreate /
# hipMemMap). bench.py, two interleaved rounds. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2; do
  for m in 1 0 2 3 4; do
    SM_TEST_OPTS=pad_alloc=$m timeout -k 10 200 $B > gpurun_out/pad2_m${m}_${i}_$T.log 2>&1 || exit 1
  done
done
