# A/B: two-row lookahead for d_{j-1} and U in the recompute-Ad pass (4096^2 and 1024^2), interleaved processes
export TMPDIR=/tmp
mkdir -p gpurun_out
SM_CGRA_LA2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "recompute or cg_vs_reference" > gpurun_out/la2_parity.log 2>&1 &&
for r in 1 2; do for v in 0 1; do
SM_CGRA_LA2=$v timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 0 --iters 60 --rounds 3 > gpurun_out/la2_${v}_$r.log 2>&1 || exit 1
SM_CGRA_LA2=$v timeout -k 10 200 python tools/tune_cg.py --n 1024 --paths recompute --xchunk 0 --iters 200 --rounds 3 > gpurun_out/la2s_${v}_$r.log 2>&1 || exit 1
done; done
