# Clocks / power of the CG pass at 8192^2 and 4096^2 (product), and of the
# stride probe's pass at 8192^2 with amd-smi sampled beside it. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/clock_probe.py --shape 8192x8192 --no-apply --chunk 20 > gpurun_out/clock8192_$T.jsonl 2> gpurun_out/clock8192_$T.err &&
timeout -k 10 200 python3 tools/clock_probe.py --shape 4096x4096 --no-apply > gpurun_out/clock4096_$T.jsonl 2> gpurun_out/clock4096_$T.err &&
( for i in $(seq 1 40); do amd-smi metric -g 0 -p -c --json > gpurun_out/smi_sp_${T}_$i.json 2>/dev/null; sleep 0.1; done ) &
timeout -k 10 120 tools/stride_probe 8192x8192 1,2 1,2 1,2 > gpurun_out/stride_8192b_$T.jsonl 2>&1
wait
