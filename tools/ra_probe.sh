# sharded recompute-Ad edge cases (Wt = 4, Wt = 2 fall-back) over the host transport
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread -k "recompute" > gpurun_out/dist_ra.log 2>&1
