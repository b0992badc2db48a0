# round 5: the coordinate-descent placement probe in the product: its tests,
# then the driver's default bench command five times (each a fresh context)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cg_paths_gpu.py -k placement > gpurun_out/r05c_tests.log 2>&1 &&
for i in 1 2 3 4 5; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r05c_bench.jsonl 2>> gpurun_out/r05c_bench.err || exit 1; done
