# round 5: the product's placement probe with repeated sweeps -- 10 contexts in
# one process, the probe test, then the driver's bench command three times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_trials.py --n 10 --hold 5 > gpurun_out/r05m_trials.jsonl 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cg_paths_gpu.py -k placement > gpurun_out/r05m_tests.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r05m_bench.jsonl 2>> gpurun_out/r05m_bench.err || exit 1; done
