# HMC timings on the device: config 1 (64^2, the recorded reference run's parameters) and 1024^2 trajectories
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/bench_configs.py --configs 2 --hmc --hmc-large 1024 > gpurun_out/hmc_times.log 2>&1
