# all-reduces on a split-off RCCL communicator: loopback / schedule tests, probe on / off
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rccl_loopback_gpu.py tests/test_cg_paths_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_splitred.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,8192x1024 --iters 100 --rounds 2 > gpurun_out/loopback_splitred1.log 2>&1 &&
SM_RCCL_SPLIT_RED=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,8192x1024 --iters 100 --rounds 2 > gpurun_out/loopback_splitred0.log 2>&1
