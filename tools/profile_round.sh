export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_stats gpurun_out/prof_fetch gpurun_out/prof_write
timeout -k 10 400 python3 bench.py > gpurun_out/bench_final.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_stats.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1
