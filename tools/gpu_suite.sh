export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/bench_v7.log 2>&1
