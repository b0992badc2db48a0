# ticketed-tail CG: one-shard + sharded parity tests, bench, loopback probe
# with the t-shard redundant scalars on / off
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py tests/test_configs_gpu.py tests/test_rccl_loopback_gpu.py tests/test_gpu_large.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_tail.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_tail.log 2>&1 &&
SM_CG_TAIL=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_notail.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x4096 > gpurun_out/loopback_tail.log 2>&1 &&
SM_CG_REDUNDANT=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024 > gpurun_out/loopback_tail_nored.log 2>&1 &&
SM_CG_TAIL=0 SM_CG_REDUNDANT=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024 > gpurun_out/loopback_notail_nored.log 2>&1
