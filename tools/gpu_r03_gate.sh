# Round 3: the GPU gate in natural test order (no multi-process-first sort),
# then the one-stream RCCL ordering against the old cross-stream build through
# the RCCL loopback (A/B/A/B). Tag $1. Outputs under gpurun_out/.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gputests_$T.log 2>&1 &&
timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_new1_$T.log 2>&1 &&
SM_LIB_PATH=tools/ab/libsm_hip_xstream.so timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_old1_$T.log 2>&1 &&
timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_new2_$T.log 2>&1 &&
SM_LIB_PATH=tools/ab/libsm_hip_xstream.so timeout -k 10 150 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_old2_$T.log 2>&1
