# t-shard Dirac apply: interior / edge split (default) against faces-first, RCCL loopback on one GPU
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x1024,4096x2048,4096x4096 --iters 50 --rounds 2 > gpurun_out/apply_split1.log 2>&1 &&
SM_APPLY_SPLIT=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x1024,4096x2048,4096x4096 --iters 50 --rounds 2 > gpurun_out/apply_split0.log 2>&1 &&
SM_EDGE_CONCURRENT=0 timeout -k 10 200 python tools/loopback_probe.py --shapes 4096x1024,4096x2048,4096x4096 --iters 50 --rounds 2 > gpurun_out/apply_conc0.log 2>&1
