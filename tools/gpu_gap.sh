# Step time against kernel time in ONE run (tag $1): bench.py under a rocprofv3
# kernel trace, then tools/step_gap.py over the timed CG passes. Outputs under
# gpurun_out/.
export TMPDIR=/tmp
T=${1:-cur}
shift
mkdir -p gpurun_out
rm -rf gpurun_out/gap_$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gap_$T -o run -- python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak "$@" > gpurun_out/gap_$T.log 2>&1 &&
python3 tools/step_gap.py $(find gpurun_out/gap_$T -name "*kernel_trace.csv" | head -1) --last 200 >> gpurun_out/gap_$T.log 2>&1
