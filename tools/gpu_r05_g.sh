# round 5: per-shard link-code choice tests; RCCL loopback timeline at 4096x512
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_gpu_parity.py -k "angle or link" > gpurun_out/r05g_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/loopback_probe.py --shapes 4096x512 --iters 200 --rounds 3 > gpurun_out/r05g_loopback.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05g_lbtrace -o run -- python -u tools/loopback_probe.py --shapes 4096x512 --iters 100 --rounds 1 > gpurun_out/r05g_lbtrace.log 2>&1
