export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python tools/small_cg.py --sizes 64,128,256,512 --paths onepass,twodir > gpurun_out/small_td.jsonl 2>&1 &&
timeout -k 10 150 python tools/tune_cg.py --n 1024 --paths onepass,twodir --xchunk 8,12,16,24 --iters 100 --rounds 3 > gpurun_out/tune1024_td.jsonl 2>&1 &&
timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths twodir --xchunk 18,32,48,64,96 --iters 30 --rounds 3 > gpurun_out/tune4096_td.jsonl 2>&1 &&
timeout -k 10 400 python tools/bench_configs.py --configs 2,3,5 --hmc > gpurun_out/configs_td.jsonl 2>&1
