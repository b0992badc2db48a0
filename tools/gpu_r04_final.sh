# Round-4 final evidence of ONE build (tag $1; every step needs the previous):
# bench.py with the driver's command (CPU baseline included), 200 steps,
# config 5, a 2-rank host-staged rehearsal (cpu_baseline beside N > 1),
# rocprofv3 kernel stats + the step gap of one bench run, FETCH / WRITE PMC.
# The gate and smoke run in tools/gpu_r04_gate.sh.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_stats_$T gpurun_out/prof_fetch_$T gpurun_out/prof_write_$T
python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/build_id_$T.txt &&
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/bench_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --config 5 --no-cpu-baseline > gpurun_out/bench_c5_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --gpus 2 --transport hosted --steps 20 --warmup 5 --no-weak > gpurun_out/bench2_hosted_$T.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats_$T -o run -- python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak > gpurun_out/prof_stats_$T.log 2>&1 &&
python3 tools/step_gap.py gpurun_out/prof_stats_$T/run_kernel_trace.csv --last 200 > gpurun_out/step_gap_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline --no-weak > gpurun_out/prof_fetch_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline --no-weak > gpurun_out/prof_write_$T.log 2>&1
