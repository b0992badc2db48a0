# Dirac apply placement probe (tools/apply_alloc_probe.py), base library
# (tools/ab/libsm_hip_base.so) and product, interleaved. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for i in 1 2; do
  SM_LIB_PATH=tools/ab/libsm_hip_base.so timeout -k 10 150 python3 tools/apply_alloc_probe.py >> gpurun_out/apply_$T.jsonl 2>> gpurun_out/apply_$T.err || exit 1
  timeout -k 10 150 python3 tools/apply_alloc_probe.py >> gpurun_out/apply_$T.jsonl 2>> gpurun_out/apply_$T.err || exit 1
done
