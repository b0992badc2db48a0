# Clocks / power under the sustained CG pass and Dirac apply (tag $1).
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
(amd-smi metric -g 0 --json > gpurun_out/smi_full_$T.json 2>&1 || true)
timeout -k 10 240 python3 tools/clock_probe.py > gpurun_out/clock_$T.jsonl 2> gpurun_out/clock_$T.err
