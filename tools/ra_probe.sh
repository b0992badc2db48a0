# paired recompute-Ad march: parity (paired default via env), timing A/B, PMC bytes
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pair_fetch
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "recompute" > gpurun_out/pair_parity.log 2>&1 &&
SM_CGRA_PAIR=1 SM_CG_FUSED=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "cg_vs_reference or pending or stepwise" > gpurun_out/pair_parity2.log 2>&1 &&
for r in 1 2; do for p in 0 1; do
SM_CGRA_PAIR=$p timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 0 --iters 60 --rounds 3 > gpurun_out/pair_${p}_$r.log 2>&1 || exit 1
done; done &&
SM_CGRA_PAIR=1 timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 16,24,32,48 --iters 40 --rounds 3 > gpurun_out/pair_x.log 2>&1 &&
SM_CGRA_PAIR=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pair_fetch -o run -- python3 tools/tune_cg.py --n 4096 --paths recompute --xchunk 0 --iters 6 --rounds 1 > gpurun_out/pair_fetch.log 2>&1
