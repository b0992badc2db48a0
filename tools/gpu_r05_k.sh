# round 5: the CG pass on buffers carved from ONE contiguous 16 GiB allocation at
# fixed offset patterns, three processes (is any pattern fast every time?)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 tools/pool_offsets 4096 3 >> gpurun_out/r05k_pool.jsonl 2>&1 || exit 1; done
