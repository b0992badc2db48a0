# even-odd CG with the ticketed tail: tests, then per-iteration time with the
# tail (default) and with the scalar kernel (SM_CG_TAIL=0) at 64^2 .. 4096^2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_eo_gpu.py tests/test_rccl_loopback_gpu.py tests/test_dist_gpu.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_eotail.log 2>&1 &&
for n in 64 256 1024 4096; do timeout -k 10 120 python tools/tune_eo.py --n $n --xchunk 0 --iters 400 --modes twodir; SM_CG_TAIL=0 timeout -k 10 120 python tools/tune_eo.py --n $n --xchunk 0 --iters 400 --modes twodir; done > gpurun_out/eo_tail.log 2>&1
