# Burst vs sustained CG throughput at 4096^2: bench.py at several step counts and
# tune_cg at several iteration counts (a clock drop under sustained fp64 load
# shows as ms per iteration growing with the run length)
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 50 200 1000; do
timeout -k 10 200 python3 bench.py --steps $k --warmup 20 --no-cpu-baseline > gpurun_out/sus_bench_$k.log 2>&1 || exit 1
done
for k in 60 200 1000; do
timeout -k 10 300 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 0 --iters $k --rounds 2 > gpurun_out/sus_tune_$k.log 2>&1 || exit 1
done
