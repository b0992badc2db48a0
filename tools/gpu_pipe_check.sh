# t-shard paths on one GPU: sharded / configs / loopback tests and the
# loopback probe (CG iteration and Dirac apply, one shard vs RCCL loopback)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_configs_gpu.py tests/test_rccl_loopback_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_pipe.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py > gpurun_out/loopback_pipe.log 2>&1 &&
SM_APPLY_EDGE_XCHUNK=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024 > gpurun_out/loopback_noedge.log 2>&1
