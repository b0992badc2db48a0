# Round 4: CG pass speed per placement rule over many contexts in one process
# (tools/alloc_trials.py), without and with held allocations. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/alloc_trials.py --modes 1,0,4 --rounds 3 > gpurun_out/trials_$T.jsonl 2> gpurun_out/trials_$T.err || exit 1
timeout -k 10 400 python3 -u tools/alloc_trials.py --modes 1,0,4 --rounds 3 --hold > gpurun_out/trials_hold_$T.jsonl 2> gpurun_out/trials_hold_$T.err || exit 1
