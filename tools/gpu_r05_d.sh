# round 5: exact link codes -- the link-code tests, the CG parity subset, config-3/5
# large tests, then bench (driver command) with the HMC-evolved figure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "link" -s > gpurun_out/r05d_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_large.py tests/test_dist_gpu.py -k "cg or angle" -s >> gpurun_out/r05d_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05d_bench.jsonl 2> gpurun_out/r05d_bench.err &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 >> gpurun_out/r05d_bench.jsonl 2>> gpurun_out/r05d_bench.err
