# Round 3: RCCL-path tests + loopback A/B (new build vs the old cross-stream
# build tools/ab/libsm_hip_xstream.so) + bench. Tag $1. Outputs under gpurun_out/.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rccl_loopback_gpu.py tests/test_cg_paths_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/looptests_$T.log 2>&1 &&
timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_new1_$T.log 2>&1 &&
SM_LIB_PATH=tools/ab/libsm_hip_xstream.so timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_old1_$T.log 2>&1 &&
timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_new2_$T.log 2>&1 &&
SM_LIB_PATH=tools/ab/libsm_hip_xstream.so timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_old2_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1
