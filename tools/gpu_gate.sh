# GPU gate of the current build (outputs under gpurun_out/, tag $1; pytest selection $2, default all -m gpu)
export TMPDIR=/tmp
T=${1:-cur}
SEL=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gputests_$T.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 &&
timeout -k 10 200 python3 bench.py --no-link-angles --no-cpu-baseline --no-weak >> gpurun_out/bench_$T.log 2>&1
