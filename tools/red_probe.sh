# recompute-Ad pass: redundant in-kernel scalars vs the scalar kernel, by lattice size (ABBA)
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for m in 0 4096 4096 0; do
i=$((i+1))
SM_CGRA_RED_MAX_BLOCKS=$m timeout -k 10 200 python tools/small_cg.py --sizes 256,512,1024,2048,4096 --paths recompute > gpurun_out/red_${m}_$i.log 2>&1 || exit 1
done
