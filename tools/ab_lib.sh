# A/B of two library builds (ab/libsm_old.so vs the in-tree one), interleaved: CG passes at 4096^2 (+ eo with $1=eo)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
for v in old new; do
if [ $v = old ]; then export SM_LIB_PATH=$PWD/ab/libsm_old.so; else unset SM_LIB_PATH; fi
timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths twodir,recompute --xchunk 0 --iters 60 --rounds 3 > gpurun_out/ab_cg_${v}_$r.log 2>&1 || exit 1
if [ "$1" = eo ]; then
timeout -k 10 200 python tools/tune_eo.py --n 4096 --modes twodir --xchunk 0 --iters 100 > gpurun_out/ab_eo_${v}_$r.log 2>&1 || exit 1
fi
done
done
