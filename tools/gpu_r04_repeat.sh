# Round 4: the driver's default bench command three times on one box (each run
# creates its own context and placement probe), for the within-box spread.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/repeat1_$T.json 2> gpurun_out/repeat1_$T.err &&
timeout -k 10 400 python3 bench.py > gpurun_out/repeat2_$T.json 2> gpurun_out/repeat2_$T.err &&
timeout -k 10 400 python3 bench.py > gpurun_out/repeat3_$T.json 2> gpurun_out/repeat3_$T.err
