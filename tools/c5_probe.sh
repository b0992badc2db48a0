# config 5's per-GPU shard at 8 GPUs (8192 x 1024 sites): recompute-Ad chunk length, via bench.py (one shard, no halo)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
for xc in 32 16 24 42; do
SM_CGRA_XCHUNK=$xc timeout -k 10 120 python3 bench.py --nx 8192 --nt-per-gpu 1024 --steps 200 --warmup 10 --applies 10 --no-cpu-baseline > gpurun_out/c5_${xc}_$r.log 2>&1 || exit 1
done
done
