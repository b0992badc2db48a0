export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_configs_gpu.py tests/test_rccl_loopback_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_pipe1.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py > gpurun_out/loopback_pipe1.log 2>&1 &&
SM_CG_FACE_PIPE=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024 > gpurun_out/loopback_nopipe1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lbtrace -o run -- python3 tools/loopback_probe.py --shapes 4096x512 --iters 50 --rounds 1 > gpurun_out/lbtrace.log 2>&1
