# round 5: planar vs site-interleaved spin planes for the CG pass's streaming shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/layout_bench 4096 64 2 > gpurun_out/r05e_layout.jsonl 2>&1 &&
timeout -k 10 120 tools/layout_bench 4096 64 3 >> gpurun_out/r05e_layout.jsonl 2>&1 &&
timeout -k 10 120 tools/layout_bench 4096 32 2 >> gpurun_out/r05e_layout.jsonl 2>&1
