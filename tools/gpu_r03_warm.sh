# Round 3: the driver's bench command (--steps 20 --warmup 5) with the Dirac
# apply sample at 100 / 400 / 1000 launches (the apply phase precedes the CG
# with no idle gap), interleaved. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for i in 1 2; do
  for n in 100 400 1000; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --applies $n --no-cpu-baseline > gpurun_out/warm_${n}_${i}_$T.log 2>&1 || exit 1
  done
done
