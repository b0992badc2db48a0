# Round 4 gate with the config-5 CG case under its band from the reference's
# own decomposition spread (manifest), then smoke.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 170 --timeout-method thread > gpurun_out/gate_$T.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
