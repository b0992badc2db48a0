# round 5: the per-buffer placement search with 3 against 6 candidates per buffer
# (trials alternate between the two in one process each, two processes)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 tools/place_buffers 4096 3 3 5 6 >> gpurun_out/r05l_m3.jsonl 2>&1 &&
  timeout -k 10 300 tools/place_buffers 4096 6 3 5 6 >> gpurun_out/r05l_m6.jsonl 2>&1 || exit 1
done
