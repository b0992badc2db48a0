# Round 4: t-shard overhead through the RCCL loopback (one shard vs the
# multi-GPU code path) at config 4's shard shapes, then a kernel trace of the
# 4096 x 512 loopback CG for the pass timeline (tools/trace_pass.py). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
rm -rf gpurun_out/lbtrace_$T
timeout -k 10 300 python3 -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 > gpurun_out/loop_$T.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lbtrace_$T -o run -- python3 tools/loopback_probe.py --shapes 4096x512 --iters 50 --rounds 1 > gpurun_out/lbtrace_$T.log 2>&1 &&
python3 tools/trace_pass.py gpurun_out/lbtrace_$T/run_kernel_trace.csv --last 30 > gpurun_out/lbtrace_$T.txt 2>&1
