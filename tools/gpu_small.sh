# One-shard scalar step by grid size: redundant scalars (<= 512 blocks,
# default) against the ticketed tail everywhere (SM_CGRA_RED_MAX_BLOCKS=0),
# plus the SURVEY configs' time to solution and the 64^2 HMC on the device.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/small_cg.py --sizes 128,256,512,1024,2048 --paths recompute --reps 3 > gpurun_out/small_red.log 2>&1 &&
SM_CGRA_RED_MAX_BLOCKS=0 timeout -k 10 300 python tools/small_cg.py --sizes 128,256,512,1024,2048 --paths recompute --reps 3 > gpurun_out/small_tail.log 2>&1 &&
timeout -k 10 300 python tools/bench_configs.py --configs 2,3 > gpurun_out/configs.log 2>&1
