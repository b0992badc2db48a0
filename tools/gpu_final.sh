# Round-end evidence on one GPU (tag $1): full GPU gate, smoke, bench (N=1),
# the multi-rank bench path on one GPU (2 ranks, host-staged halos), config 5
# time to solution, rocprof stats + FETCH/WRITE PMC, and the t-shard overhead
# through the RCCL loopback (redundant t-shard scalars on / off). Outputs under
# gpurun_out/.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_stats_$T gpurun_out/prof_fetch_$T gpurun_out/prof_write_$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_$T.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 2 --transport hosted --steps 50 --warmup 10 --no-weak > gpurun_out/bench2_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench_c5_$T.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats_$T -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_stats_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline > gpurun_out/prof_fetch_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline > gpurun_out/prof_write_$T.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x4096 --iters 100 --rounds 2 > gpurun_out/loopback_$T.log 2>&1 &&
SM_CG_RED_SHARDS=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 100 --rounds 2 > gpurun_out/loopback_nored_$T.log 2>&1
