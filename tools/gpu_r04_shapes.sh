# Round 4: recompute-Ad pass launch shapes at 4096^2 on one context (so one
# placement, the probe's choice), interleaved (tools/tune_shapes.py). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:1,32,1 4096x4096:2,64,1 4096x4096:1,128,1 4096x4096:2,32,1 4096x4096:4,32,1 4096x4096:1,64,1 --iters 100 --rounds 4 > gpurun_out/shapes_$T.log 2>&1 || exit 1
