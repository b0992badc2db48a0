# rocprof kernel durations of the one-pass even-odd CG at 4096^2: ab/libsm_old.so vs in-tree (old, new, new, old)
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in old new new old; do
i=$((i+1))
if [ $v = old ]; then export SM_LIB_PATH=$PWD/ab/libsm_old.so; else unset SM_LIB_PATH; fi
rm -rf gpurun_out/eop_${v}_$i
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eop_${v}_$i -o run -- python3 tools/tune_eo.py --n 4096 --modes twodir --xchunk 0 --iters 100 > gpurun_out/eop_${v}_$i.log 2>&1 || exit 1
done
