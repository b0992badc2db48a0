# Round 4: placement rules 5 (>= 2 GiB + contiguous), 6 (>= 1 GiB +
# contiguous), 7 (one contiguous pool), 1 (>= 2 GiB) over many contexts, two
# processes with held allocations (tools/alloc_trials.py; the first use of
# this script, tag t2, ran rules 1, 2, 3, 5). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for p in 1 2; do
  timeout -k 10 400 python3 -u tools/alloc_trials.py --modes 5,6,7,1 --rounds 3 --hold > gpurun_out/trials3_${p}_$T.jsonl 2> gpurun_out/trials3_${p}_$T.err || exit 1
done
