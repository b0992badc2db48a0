# Round 3: bench.py with the driver's command (--steps 20 --warmup 5) and the
# default 200 steps, after the no-idle reordering of the CG setup. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/drv${i}_$T.log 2>&1 || exit 1
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/drvdef_$T.log 2>&1
