# recompute-Ad chunk length at 4096^2, interleaved rounds (block-round shapes: 32 rows = 4.75 rounds of 512 blocks, 39 = 3.9, 52 = 2.9, 78 = 1.97)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 300 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 32,39,52,78 --iters 300 --rounds 4 > gpurun_out/chunk_$r.log 2>&1 || exit 1
done
