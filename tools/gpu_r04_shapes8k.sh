# Round 4: recompute-Ad pass launch shapes at 8192^2 (config 5) on one context
# (one placement, the probe's choice), interleaved (tools/tune_shapes.py). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/tune_shapes.py 8192x8192:4,32,1 8192x8192:1,64,1 8192x8192:1,32,1 8192x8192:2,32,1 8192x8192:4,64,1 8192x8192:2,64,1 8192x8192:1,128,1 --iters 40 --rounds 4 > gpurun_out/shapes8k_$T.log 2>&1 || exit 1
