# A subset of the GPU gate, verbose and streaming: bash tools/gpu_subset.sh <tag> <pytest args...>
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 170 --timeout-method thread "$@" > gpurun_out/subset_$T.log 2>&1
