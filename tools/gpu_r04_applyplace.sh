# Round 4: is the Dirac apply placement-sensitive? 8 candidate (in, out)
# pairs per process, contiguous 2 GiB and own-size allocations, two processes
# each (tools/apply_place_trials.py). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for m in contig2g own contig2g own; do
  timeout -k 10 200 python3 -u tools/apply_place_trials.py --pairs 8 --mode $m >> gpurun_out/applyplace_$T.jsonl 2>> gpurun_out/applyplace_$T.err || exit 1
done
