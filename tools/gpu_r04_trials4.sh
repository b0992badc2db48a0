# Round 4: placement rules without the probe -- 5 (>= 2 GiB contiguous, the
# default), 8 (one contiguous pool of 2 GiB slots), 1 (>= 2 GiB plain) --
# then rule 5 with the probe, over many contexts per process with held
# allocations (tools/alloc_trials.py). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/alloc_trials.py --modes 5,8,1 --rounds 3 --hold > gpurun_out/trials4_a_$T.jsonl 2> gpurun_out/trials4_a_$T.err || exit 1
timeout -k 10 400 python3 -u tools/alloc_trials.py --modes 5,8 --rounds 3 --hold --probe 5 > gpurun_out/trials4_b_$T.jsonl 2> gpurun_out/trials4_b_$T.err || exit 1
