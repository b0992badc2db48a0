# Rest of a GPU round once the test gate is known green: selected tests, smoke,
# bench, CG tune, rocprof stats + FETCH/WRITE PMC, apply sweep, loopback probe
# (outputs under gpurun_out/, tag $1; pytest selection $2)
export TMPDIR=/tmp
T=${1:-cur}
SEL=${2:-tests/test_rccl_loopback_gpu.py}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_stats_$T gpurun_out/prof_fetch_$T gpurun_out/prof_write_$T
timeout -k 10 300 python -u -m pytest $SEL -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_$T.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats_$T -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_stats_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline > gpurun_out/prof_fetch_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline > gpurun_out/prof_write_$T.log 2>&1 &&
timeout -k 10 200 python tools/tune_dslash.py --bt 64,256 --xchunk 32,64,128,256 --remap 0,1 --variant 1,2 --rounds 3 > gpurun_out/tune_dslash_$T.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py > gpurun_out/loopback_$T.log 2>&1
