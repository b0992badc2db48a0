export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "recompute or pending or stepwise" > gpurun_out/ra_parity.log 2>&1 &&
timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths twodir,recompute --xchunk 0 --iters 30 --rounds 3 > gpurun_out/ra_tune4096_f1.log 2>&1 &&
SM_CGRA_FOLD=0 timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 0,24,32,48,64 --iters 30 --rounds 3 > gpurun_out/ra_tune4096_f0.log 2>&1 &&
timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 16,24,32,48,64,96 --iters 30 --rounds 3 > gpurun_out/ra_tune4096_x.log 2>&1 &&
timeout -k 10 200 python tools/tune_cg.py --n 1024 --paths twodir,recompute --xchunk 0,8,12,16,24,32 --iters 50 --rounds 3 > gpurun_out/ra_tune1024.log 2>&1
