# recompute-Ad launch shape re-check at the shard shapes (power-of-two chunk lengths)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_shapes.py --iters 200 --rounds 3 8192x8192:4,32,1 8192x8192:1,32,1 8192x8192:2,32,1 8192x8192:4,16,1 > gpurun_out/reshape_b.log 2>&1 &&
timeout -k 10 300 python tools/tune_shapes.py --iters 400 --rounds 3 4096x512:1,48,0 4096x512:1,32,0 4096x512:1,64,0 4096x1024:1,40,1 4096x1024:1,32,1 4096x1024:1,64,1 4096x2048:1,32,1 4096x2048:1,64,1 8192x1024:1,40,1 8192x1024:1,32,1 8192x1024:1,64,1 2048x2048:1,40,0 2048x2048:1,32,0 2048x2048:1,64,0 > gpurun_out/reshape_c.log 2>&1
