# SURVEY §8d config timings with the library defaults (tag = $1), JSON lines in gpurun_out/configs_$1.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python tools/bench_configs.py --configs 2,3,5 --hmc --hmc-large 1024 --tag "$1" > gpurun_out/configs_$1.jsonl 2>gpurun_out/configs_$1.err &&
timeout -k 10 150 python tools/small_cg.py --sizes 64,128,256,512,1024 --paths twodir,recompute > gpurun_out/small_$1.jsonl 2>&1
