# Round 4: quick check of a rebuilt library -- the placement tests, the CG
# paths at small sizes, smoke and one bench run. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cg_paths_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/quick_tests_$T.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/quick_smoke_$T.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak > gpurun_out/quick_bench_$T.log 2>&1
