set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/place_buffers 4096 8 5 5 > gpurun_out/r05a_place1.jsonl 2>&1 &&
timeout -k 10 120 tools/place_buffers 4096 8 5 5 > gpurun_out/r05a_place2.jsonl 2>&1 &&
timeout -k 10 120 tools/place_buffers 4096 8 5 0 > gpurun_out/r05a_place0.jsonl 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_configs_gpu.py tests/test_gpu_large.py -k 8192 -s > gpurun_out/r05a_c5tests.log 2>&1
