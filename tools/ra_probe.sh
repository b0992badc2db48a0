# recompute-Ad pass with the shared h1 products: parity subset, timing A/B against the stored-Ad pass
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/h1_stats
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "cg or large_lattice" > gpurun_out/h1_parity.log 2>&1 &&
timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute,twodir --xchunk 0 --iters 60 --rounds 3 > gpurun_out/h1_tune.log 2>&1 &&
timeout -k 10 200 python tools/tune_cg.py --n 1024 --paths recompute,twodir --xchunk 0 --iters 200 --rounds 3 > gpurun_out/h1_tune1024.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h1_stats -o run -- python3 tools/tune_cg.py --n 4096 --paths recompute --xchunk 32 --iters 30 --rounds 1 > gpurun_out/h1_stats.log 2>&1
