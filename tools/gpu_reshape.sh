# recompute-Ad launch shape re-check after the ticketed tail and the x row parity
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_shapes.py --iters 200 --rounds 3 4096x4096:1,32,1 4096x4096:1,48,1 4096x4096:1,64,1 4096x4096:1,80,1 4096x4096:1,96,1 4096x4096:1,128,1 4096x4096:2,32,1 4096x4096:2,64,1 4096x4096:4,32,1 4096x4096:4,48,1 > gpurun_out/reshape4096.log 2>&1 &&
timeout -k 10 300 python tools/tune_shapes.py --iters 100 --rounds 3 8192x8192:4,48,1 8192x8192:4,32,1 8192x8192:4,64,1 8192x8192:1,48,1 8192x8192:1,64,1 8192x8192:1,96,1 > gpurun_out/reshape8192.log 2>&1
