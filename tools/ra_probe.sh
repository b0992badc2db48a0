# recompute-Ad CG pass: waves-per-block x chunk sweep at 4096^2 and 2048^2/1024^2
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 4 2 1; do
  SM_CGRA_WPB=$w timeout -k 10 200 python tools/tune_cg.py --n 4096 --paths recompute --xchunk 24,32,48,64,96,128 --iters 30 --rounds 3 > gpurun_out/ra_wpb${w}_4096.log 2>&1 || exit 1
done
for w in 4 2; do
  SM_CGRA_WPB=$w timeout -k 10 200 python tools/tune_cg.py --n 2048 --paths recompute --xchunk 12,16,24,32 --iters 60 --rounds 3 > gpurun_out/ra_wpb${w}_2048.log 2>&1 || exit 1
  SM_CGRA_WPB=$w timeout -k 10 200 python tools/tune_cg.py --n 1024 --paths recompute --xchunk 8,12,16,24 --iters 100 --rounds 3 > gpurun_out/ra_wpb${w}_1024.log 2>&1 || exit 1
done
