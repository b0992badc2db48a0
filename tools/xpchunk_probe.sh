# recompute-Ad pass at 4096^2: chunk length of the x-updating (even) passes, odd passes at 32 rows; ABBA via bench.py (sustained)
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for xx in 32 64 64 32 32 48 48 32; do
i=$((i+1))
SM_CGRA_XCHUNK_X=$xx timeout -k 10 120 python3 bench.py --steps 200 --warmup 10 --applies 10 --no-cpu-baseline > gpurun_out/xpc_${xx}_$i.log 2>&1 || exit 1
done
