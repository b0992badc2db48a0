# recompute-Ad pass: fold 1 (exact folded bracket) vs fold 2 (fused multiply-adds), ABBA order, long runs at 4096^2
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for f in 1 2 2 1 1 2 2 1; do
i=$((i+1))
SM_CGRA_FOLD=$f timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 0 --iters 400 --rounds 2 > gpurun_out/ab_fold${f}_$i.log 2>&1 || exit 1
done
