# config 4/5 tests at full size and the config 5 time to solution on one GPU
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_configs_gpu.py tests/test_cg_paths_gpu.py -m gpu -x -v -s --timeout 250 --timeout-method thread > gpurun_out/gputests_c5.log 2>&1 &&
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench_c5.log 2>&1
