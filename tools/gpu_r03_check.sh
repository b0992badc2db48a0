# Re-entry check of a rebuilt tree (tag $1): full GPU gate in natural order,
# smoke, and bench.py with the driver's command. Outputs under gpurun_out/.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gputests_$T.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$T.log 2>&1
