# Round-4 end-of-round evidence of ONE build in one call (tag $1): the GPU
# gate in natural order, smoke, then tools/gpu_r04_final.sh (benches incl.
# the driver's command and a 2-rank hosted line, kernel stats, step gap,
# FETCH / WRITE PMC).
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gate_$T.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 &&
bash tools/gpu_r04_final.sh $T
