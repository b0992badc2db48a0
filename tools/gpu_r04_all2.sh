# Round 4 end evidence (tag $1) while the config-5 bar waits for the
# reference's own decomposition spread: the gate without that one case, smoke,
# then tools/gpu_r04_final.sh (benches, kernel stats, step gap, PMC).
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 170 --timeout-method thread --deselect "tests/test_gpu_large.py::test_cg_matches_reference[l8192x8192_b2_m-0p19]" > gpurun_out/gate_$T.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 &&
bash tools/gpu_r04_final.sh $T
