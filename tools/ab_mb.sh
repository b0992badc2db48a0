# recompute-Ad pass at 4096^2: one-block vs 8-block scalar reduction (SM_CG_SCALAR_MB_MIN), ABBA bench.py + rocprof
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for m in 1000000 2048 2048 1000000 1000000 2048; do
i=$((i+1))
SM_CG_SCALAR_MB_MIN=$m timeout -k 10 120 python3 bench.py --steps 200 --warmup 10 --applies 10 --no-cpu-baseline > gpurun_out/mb_${m}_$i.log 2>&1 || exit 1
done
rm -rf gpurun_out/mbp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mbp -o run -- python3 bench.py --steps 50 --warmup 5 --applies 10 --no-cpu-baseline > gpurun_out/mbp.log 2>&1
