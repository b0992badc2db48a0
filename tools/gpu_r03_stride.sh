# Allocation layouts of the CG pass's streams (tools/stride_probe.hip),
# interleaved in one process. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 280 tools/stride_probe 4096x4096 1,2,0,3 1,2,0,2,8 1,2,0,1,8 1,2 1,2,0,3 1,2,0,2,8 1,2,0,1,8 1,2 1,2,0,3 1,2,0,2,8 1,2,0,1,8 1,2 1,2,0,3 1,2,0,2,8 1,2,0,1,8 > gpurun_out/stride_4096_$T.jsonl 2>&1
