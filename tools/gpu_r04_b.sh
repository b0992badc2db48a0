# Round 4: the link-code and parity tests after the pre-scaled-links merge,
# the link-code toggle on 2 t-shards, then the allocation-size counters
# (tools/gpu_r04_alloc.sh). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_cg_paths_gpu.py tests/test_gpu_large.py -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/b_tests_$T.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -k link_angle -x -v --timeout 120 --timeout-method thread > gpurun_out/b_dist_tests_$T.log 2>&1 || exit 1
bash tools/gpu_r04_alloc.sh $T
