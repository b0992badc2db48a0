# recompute-Ad launch shapes at 1024^2 (config 2) and 2048^2 with link angles
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_shapes.py --iters 400 --rounds 3 1024x1024:4,12,0 1024x1024:4,16,0 1024x1024:4,8,0 1024x1024:1,16,0 1024x1024:1,32,0 1024x1024:2,16,0 1024x1024:1,8,0 2048x2048:1,64,1 2048x2048:1,40,1 2048x2048:1,32,1 2048x2048:4,16,1 > gpurun_out/reshape_d.log 2>&1
