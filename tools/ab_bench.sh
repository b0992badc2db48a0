# A/B of two library builds on bench.py (ab/libsm_old.so vs in-tree), ABBA, plus rocprof kernel stats of each
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in old new new old; do
i=$((i+1))
if [ $v = old ]; then export SM_LIB_PATH=$PWD/ab/libsm_old.so; else unset SM_LIB_PATH; fi
timeout -k 10 120 python3 bench.py --steps 200 --warmup 10 --applies 10 --no-cpu-baseline > gpurun_out/abb_${v}_$i.log 2>&1 || exit 1
done
for v in old new; do
if [ $v = old ]; then export SM_LIB_PATH=$PWD/ab/libsm_old.so; else unset SM_LIB_PATH; fi
rm -rf gpurun_out/abp_$v
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abp_$v -o run -- python3 bench.py --steps 50 --warmup 5 --applies 10 --no-cpu-baseline > gpurun_out/abp_$v.log 2>&1 || exit 1
done
