# Round 4: placement probe (8 candidates, the default) against none, three
# interleaved bench.py pairs on whichever box this lands on. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak"
for i in 1 2 3; do
  SM_TEST_OPTS=place_probe=1 timeout -k 10 200 $B > gpurun_out/probe3_k1_${i}_$T.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/probe3_k8_${i}_$T.log 2>&1 || exit 1
done
