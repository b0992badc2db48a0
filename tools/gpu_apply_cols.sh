# t-shard Dirac apply with the edge-column kernel: sharded / loopback / configs
# tests, then the loopback probe with it (default) and without (SM_APPLY_EDGE_COLS=0)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_rccl_loopback_gpu.py tests/test_dist_gpu.py tests/test_configs_gpu.py tests/test_dropin_gpu.py tests/test_md_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_cols.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048,4096x4096 --iters 50 --rounds 2 > gpurun_out/apply_cols1.log 2>&1 &&
SM_APPLY_EDGE_COLS=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048,4096x4096 --iters 50 --rounds 2 > gpurun_out/apply_cols0.log 2>&1
