# recompute-Ad pass: one-wave blocks with one-round chunk lengths (4096^2: 74 waves x XB blocks, 2048 wave slots)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 32 --iters 60 --rounds 3 > gpurun_out/w1_base_$r.log 2>&1 || exit 1
SM_CGRA_WPB=1 timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 152,160,171,205 --iters 60 --rounds 3 > gpurun_out/w1_long_$r.log 2>&1 || exit 1
done
