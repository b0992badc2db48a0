# Round 4: config 5 against the reference's fixture through every CG path
# (tools/c5_paths.py). Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/c5_paths.py > gpurun_out/c5paths_$T.log 2>&1 || exit 1
