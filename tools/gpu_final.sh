# Round-end evidence on one GPU (tag $1): full GPU gate (natural order), smoke,
# bench (N=1, the driver's command and the 200-step default), the multi-rank
# bench path on one GPU (2 ranks, host-staged halos), config 5 time to
# solution, rocprof kernel trace + stats (with the step-vs-kernel gap of the
# timed CG passes), FETCH/WRITE PMC passes, and the t-shard overhead through
# the RCCL loopback. Outputs under gpurun_out/; summarise with
#   python tools/summarize_prof.py --round r03 --tag _final --suffix _$T
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_stats_$T gpurun_out/prof_fetch_$T gpurun_out/prof_write_$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gputests_$T.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 2 --transport hosted --steps 50 --warmup 10 --no-weak > gpurun_out/bench2_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench_c5_$T.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats_$T -o run -- python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak > gpurun_out/prof_stats_$T.log 2>&1 &&
python3 tools/step_gap.py gpurun_out/prof_stats_$T/run_kernel_trace.csv --last 200 > gpurun_out/step_gap_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline --no-weak > gpurun_out/prof_fetch_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline --no-weak > gpurun_out/prof_write_$T.log 2>&1 &&
timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x4096 --iters 100 --rounds 2 > gpurun_out/loopback_$T.log 2>&1
