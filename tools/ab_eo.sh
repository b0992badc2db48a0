# A/B of two library builds on the one-pass even-odd CG at 4096^2 (ab/libsm_old.so vs in-tree), interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
for v in old new; do
if [ $v = old ]; then export SM_LIB_PATH=$PWD/ab/libsm_old.so; else unset SM_LIB_PATH; fi
timeout -k 10 200 python tools/tune_eo.py --n 4096 --modes twodir --xchunk 0,8 --iters 100 > gpurun_out/ab_eo_${v}_$r.log 2>&1 || exit 1
done
done
