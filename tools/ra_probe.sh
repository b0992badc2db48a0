# scalar-kernel latency after batching the partial loads: kernel stats of a 4096^2 CG run
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/sc_stats
timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute,twodir --xchunk 0 --iters 60 --rounds 3 > gpurun_out/sc_tune.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sc_stats -o run -- python3 tools/tune_cg.py --n 4096 --paths recompute --xchunk 32 --iters 30 --rounds 1 > gpurun_out/sc_stats.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "cg" > gpurun_out/sc_parity.log 2>&1
