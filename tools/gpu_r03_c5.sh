# Round 3: config 5 (8192^2 solve to 1e-10, m0 = -0.19) under the three march
# schedules of the recompute-Ad pass, interleaved. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for r in 1 2 1 2 1 2; do
  SM_TEST_OPTS=rev=$r timeout -k 10 200 python3 bench.py --config 5 >> gpurun_out/c5_rev_$T.log 2>&1 || exit 1
done
