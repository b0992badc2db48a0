# round 5: t-shard overheads on the RCCL loopback: host
# enqueue time per CG pass, the parallel face pack, the apply's interior/edge
# split with narrower t-blocks; then the t-shard parity tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r05j_*
L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 3"
timeout -k 10 300 $L > gpurun_out/r05j_default.log 2>&1 &&
SM_TEST_OPTS=bt=64,apply_split=1 timeout -k 10 300 $L > gpurun_out/r05j_bt64_split.log 2>&1 &&
SM_TEST_OPTS=bt=128,apply_split=1 timeout -k 10 300 $L > gpurun_out/r05j_bt128_split.log 2>&1 &&
SM_TEST_OPTS=bt=64 timeout -k 10 300 $L > gpurun_out/r05j_bt64.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05j_lbtrace -o run -- python -u tools/loopback_probe.py --shapes 4096x512 --iters 100 --rounds 1 > gpurun_out/r05j_lbtrace.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_rccl_loopback_gpu.py tests/test_md_gpu.py > gpurun_out/r05j_tests.log 2>&1
