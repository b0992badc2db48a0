set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 tools/place_buffers 4096 3 3 5 6 > gpurun_out/r05b_descent5a.jsonl 2>&1 &&
timeout -k 10 180 tools/place_buffers 4096 3 3 0 6 > gpurun_out/r05b_descent0a.jsonl 2>&1 &&
timeout -k 10 180 tools/place_buffers 4096 3 3 5 6 > gpurun_out/r05b_descent5b.jsonl 2>&1 &&
timeout -k 10 180 tools/place_buffers 4096 3 3 0 6 > gpurun_out/r05b_descent0b.jsonl 2>&1
