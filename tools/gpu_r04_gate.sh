# Round 4: the whole GPU gate in natural order, smoke, then interleaved
# bench.py pairs of the default placement (pad_alloc 5: >= 2 GiB contiguous)
# against the round-3 rule (pad_alloc 1). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gate_$T.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || exit 1
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2 3; do
  SM_TEST_OPTS=pad_alloc=1 timeout -k 10 200 $B > gpurun_out/gate_pad1_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/gate_pad5_${i}_$T.log 2>&1 || exit 1
done
