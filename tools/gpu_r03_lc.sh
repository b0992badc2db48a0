# Round 3: one-double link codes (sm_linkcode.h) against the angle form of the
# previous build (tools/ab/libsm_hip_base.so): rocprofv3 kernel durations of the
# CG pass in interleaved bench.py runs, then the complex-vs-codes pass time per
# shard shape (tools/link_probe.py). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2; do
  rm -rf gpurun_out/lcprof_base_${i}_$T gpurun_out/lcprof_new_${i}_$T
  SM_LIB_PATH=tools/ab/libsm_hip_base.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lcprof_base_${i}_$T -o run -- $B > gpurun_out/lcprof_base_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lcprof_new_${i}_$T -o run -- $B > gpurun_out/lcprof_new_${i}_$T.log 2>&1 || exit 1
done
timeout -k 10 400 python3 tools/link_probe.py > gpurun_out/link_probe_$T.log 2>&1
