# face packs in 64-thread blocks: sharded / loopback tests, loopback probe
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_rccl_loopback_gpu.py tests/test_dist_gpu.py tests/test_cg_paths_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_pack64.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,8192x1024 --iters 100 --rounds 2 > gpurun_out/loopback_pack64.log 2>&1
