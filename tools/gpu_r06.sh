# Round-6 GPU experiments, one function per experiment; run ONE per gpurun call:
#   gpurun -- 'bash tools/gpu_r06.sh <name> [tag]'
# Outputs land in gpurun_out/r06<x>_*; the summaries kept are profiles/r06_<x>_*.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out

# a: one communicator on one comm stream -- the RCCL loopback and hosted
#    t-shard tests, the loopback's per-iteration time at 4096x512 / 1024, and the bench
a() {
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/r06a_build_id.txt &&
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    tests/test_dist_gpu.py -k "loopback or sharded_gpu_path or recompute" > gpurun_out/r06a_tests.log 2>&1 &&
  timeout -k 10 300 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 3 \
    > gpurun_out/r06a_loopback.log 2>&1 &&
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06a_bench.log 2>&1 &&
  timeout -k 10 300 python3 bench.py --gpus 2 --transport hosted --steps 20 --warmup 5 --no-weak \
    > gpurun_out/r06a_bench2.log 2>&1
}

# b: the RCCL stream A/B on the loopback (rccl_main=1 main stream, 0 comm stream with event hops),
#    twice each, then the loopback / t-shard tests on the default
b() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 20"
  for i in 1 2; do
    for m in 1 0; do
      SM_TEST_OPTS=rccl_main=$m timeout -k 10 300 $L > gpurun_out/r06b_main${m}_$i.log 2>&1 || return 1
    done
    # round 5's two communicators (tools/ab_libs/libsm_hip_r05.so, built from the round-5 head)
    SM_LIB_PATH=$PWD/tools/ab_libs/libsm_hip_r05.so SM_LIB_AB=1 timeout -k 10 300 $L > gpurun_out/r06b_r05_$i.log 2>&1 || return 1
  done
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    tests/test_dist_gpu.py tests/test_gpu_parity.py -k "loopback or sharded_gpu_path or recompute or link" \
    > gpurun_out/r06b_tests.log 2>&1
}

# gate: the full GPU gate in natural order, then smoke (tag $1)
gate() {
  local T=${1:-cur}
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/build_id_$T.txt &&
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gate_$T.log 2>&1 &&
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
}

"$@"
