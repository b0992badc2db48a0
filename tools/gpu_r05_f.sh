# round 5: packed flag nibbles -- link-code tests (one shard + loopback), t-shard link tests, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "link" -s > gpurun_out/r05f_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_large.py tests/test_dist_gpu.py tests/test_cg_paths_gpu.py -k "cg or angle or tshard" -s >> gpurun_out/r05f_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05f_bench.jsonl 2> gpurun_out/r05f_bench.err &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 >> gpurun_out/r05f_bench.jsonl 2>> gpurun_out/r05f_bench.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r05f_bench.jsonl 2>> gpurun_out/r05f_bench.err
