# Allocation layouts of the CG pass's streams at the t-shard shapes
# (tools/stride_probe.hip), interleaved per shape. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for s in 4096x2048 4096x1024 4096x512 2048x2048 1024x1024; do
  timeout -k 10 100 tools/stride_probe $s 1,2 1,2,0,1,8 1,2 1,2,0,1,8 1,2,0,1 1,2,0,1,8 >> gpurun_out/stride_shapes_$T.jsonl 2>&1 || exit 1
done
