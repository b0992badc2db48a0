# Round 4: does the placement probe pay on the t-shard shapes of config 4
# (4096 x 2048 / 1024 / 512 per GPU)? One-GPU bench.py on those shapes,
# probe off vs on (probe_min_mib lowered so the smaller fields are probed),
# interleaved. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for nt in 2048 1024 512; do
  B="python3 bench.py --nx 4096 --nt $nt --steps 400 --warmup 40 --applies 20 --no-cpu-baseline --no-weak"
  for i in 1 2; do
    SM_TEST_OPTS=place_probe=1 timeout -k 10 200 $B > gpurun_out/psmall_${nt}_off_${i}_$T.log 2>&1 || exit 1
    SM_TEST_OPTS=probe_min_mib=32 timeout -k 10 200 $B > gpurun_out/psmall_${nt}_on_${i}_$T.log 2>&1 || exit 1
  done
done
