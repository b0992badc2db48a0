# interior/edge split of t-shards measured on ONE shard (SM_SPLIT_TEST: 0 none, 1 edge after interior, 2 concurrent)
export TMPDIR=/tmp
mkdir -p gpurun_out
SM_SPLIT_TEST=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "cg_vs_reference and (recompute or twodir) or large_lattice or pending" > gpurun_out/split_parity.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/split_dist.log 2>&1 &&
for r in 1 2; do for m in 0 1 2; do
SM_SPLIT_TEST=$m timeout -k 10 200 python3 bench.py --steps 60 --warmup 6 --applies 40 --no-cpu-baseline > gpurun_out/split_bench_${m}_$r.log 2>&1 || exit 1
done; done
