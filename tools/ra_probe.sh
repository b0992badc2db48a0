# even-odd suite with the one-pass eo CG as default (incl. sharded = six-launch fall-back), HMC timing
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_eo_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread -k "eo or even_odd" > gpurun_out/eotd_def.log 2>&1 &&
timeout -k 10 400 python tools/bench_configs.py --configs "" --hmc --hmc-large 1024 --tag "eotd" > gpurun_out/eotd_hmc.jsonl 2>gpurun_out/eotd_hmc.err &&
timeout -k 10 300 python tools/tune_eo.py --n 256 --xchunk 0,1,2,3 --iters 400 --modes twodir > gpurun_out/eotd_256b.log 2>&1
