# A/B of two library builds on the one-pass even-odd CG at 4096^2 (ab/libsm_old.so vs in-tree), ABBA order
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in old new new old old new; do
i=$((i+1))
if [ $v = old ]; then export SM_LIB_PATH=$PWD/ab/libsm_old.so; else unset SM_LIB_PATH; fi
timeout -k 10 200 python tools/tune_eo.py --n 4096 --modes twodir --xchunk 0 --iters 200 > gpurun_out/ab_eo_${v}_$i.log 2>&1 || exit 1
done
