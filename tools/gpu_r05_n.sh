# round 5: t-shard comm stream at the highest priority (edge launches + faces) vs default, loopback A/B/A/B
set -o pipefail
mkdir -p gpurun_out
L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3"
for r in 1 2; do
  timeout -k 10 300 $L > gpurun_out/r05n_default_$r.log 2>&1 &&
  SM_TEST_OPTS=comm_prio=1 timeout -k 10 300 $L > gpurun_out/r05n_prio_$r.log 2>&1 || exit 1
done
