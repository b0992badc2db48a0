# round 5: the full GPU gate in natural order, then smoke (tag $1)
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/build_id_$T.txt &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gate_$T.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
