# Round-5 GPU experiments, one function per experiment; run ONE per gpurun call:
#   gpurun -- 'bash tools/gpu_r05.sh <name>'
# Outputs land in gpurun_out/r05<x>_*; the summaries kept are profiles/r05_<x>_*.
# Binaries (tools/place_buffers, layout_bench, pool_offsets) are built on the dev
# host first (their headers give the hipcc lines).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out

# a: which streamed buffer carries the CG pass's placement state (one-buffer
#    substitutions, two processes with >= 2 GiB contiguous, one own-size), then
#    config 5 over 8 t-shards against the reference fixture
a() {
  timeout -k 10 120 tools/place_buffers 4096 8 5 5 > gpurun_out/r05a_place1.jsonl 2>&1 &&
  timeout -k 10 120 tools/place_buffers 4096 8 5 5 > gpurun_out/r05a_place2.jsonl 2>&1 &&
  timeout -k 10 120 tools/place_buffers 4096 8 5 0 > gpurun_out/r05a_place0.jsonl 2>&1 &&
  timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_configs_gpu.py \
    tests/test_gpu_large.py -k 8192 -s > gpurun_out/r05a_c5tests.log 2>&1
}

# b: the per-buffer search (descent) in the tool, 6 trials x 2 processes per allocation rule
b() {
  for m in 5 0 5 0; do
    timeout -k 10 180 tools/place_buffers 4096 3 3 $m 6 >> gpurun_out/r05b_descent$m.jsonl 2>&1 || return 1
  done
}

# c: the product probe's tests, then the driver's bench command five times
c() {
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cg_paths_gpu.py \
    -k placement > gpurun_out/r05c_tests.log 2>&1 || return 1
  for i in 1 2 3 4 5; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r05c_bench.jsonl 2>> gpurun_out/r05c_bench.err || return 1
  done
}

# d/f: exact link codes (d: 16-bit flag words; f: packed flag nibbles) -- link tests,
#      CG parity, config 3/5 large tests, t-shard link tests, bench with the evolved field
f() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "link" -s > gpurun_out/r05f_tests.log 2>&1 &&
  timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_large.py \
    tests/test_dist_gpu.py tests/test_cg_paths_gpu.py -k "cg or angle or tshard" -s >> gpurun_out/r05f_tests.log 2>&1 &&
  for a in "--steps 20 --warmup 5" "--steps 200 --warmup 20" "--steps 20 --warmup 5"; do
    timeout -k 10 300 python -u bench.py $a >> gpurun_out/r05f_bench.jsonl 2>> gpurun_out/r05f_bench.err || return 1
  done
}

# e: planar vs site-interleaved spin planes for the CG pass's streaming shape
e() {
  timeout -k 10 120 tools/layout_bench 4096 64 2 > gpurun_out/r05e_layout.jsonl 2>&1 &&
  timeout -k 10 120 tools/layout_bench 4096 64 3 >> gpurun_out/r05e_layout.jsonl 2>&1 &&
  timeout -k 10 120 tools/layout_bench 4096 32 2 >> gpurun_out/r05e_layout.jsonl 2>&1
}

# g: per-shard link-code choice tests; RCCL loopback at 4096x512
g() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py \
    tests/test_gpu_parity.py -k "angle or link" > gpurun_out/r05g_tests.log 2>&1 &&
  timeout -k 10 300 python -u tools/loopback_probe.py --shapes 4096x512 --iters 200 --rounds 3 > gpurun_out/r05g_loopback.log 2>&1
}

# h: loopback kernel timeline + apply split A/B; the CG pass's L2 / fabric
#    counters per march schedule and tile order, with timing pairs
h() {
  rm -rf gpurun_out/r05h_*
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05h_lbtrace -o run -- python -u \
    tools/loopback_probe.py --shapes 4096x512 --iters 100 --rounds 1 > gpurun_out/r05h_lbtrace.log 2>&1 || return 1
  local P="python3 bench.py --steps 10 --warmup 2 --applies 4 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  local B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  for v in default rev=1 rev=0 ra_remap=0; do
    if [ $v = default ]; then unset SM_TEST_OPTS; else export SM_TEST_OPTS=$v; fi
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
      -d gpurun_out/r05h_pmc_$v -o run -- $P > gpurun_out/r05h_pmc_$v.log 2>&1 || return 1
    timeout -k 10 200 $B > gpurun_out/r05h_bench_$v.log 2>&1 || return 1
  done
  unset SM_TEST_OPTS
}

# j: t-shard overheads on the loopback: host enqueue time, apply split with narrower t-blocks
j() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 3"
  timeout -k 10 300 $L > gpurun_out/r05j_default.log 2>&1 &&
  SM_TEST_OPTS=bt=64,apply_split=1 timeout -k 10 300 $L > gpurun_out/r05j_bt64_split.log 2>&1 &&
  SM_TEST_OPTS=bt=128,apply_split=1 timeout -k 10 300 $L > gpurun_out/r05j_bt128_split.log 2>&1 &&
  SM_TEST_OPTS=bt=64 timeout -k 10 300 $L > gpurun_out/r05j_bt64.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05j_lbtrace -o run -- python -u \
    tools/loopback_probe.py --shapes 4096x512 --iters 100 --rounds 1 > gpurun_out/r05j_lbtrace.log 2>&1
}

# k: the CG pass on buffers carved from one contiguous 16 GiB allocation at fixed offset patterns
k() {
  for i in 1 2 3; do timeout -k 10 120 tools/pool_offsets 4096 3 >> gpurun_out/r05k_pool.jsonl 2>&1 || return 1; done
}

# l: the tool's per-buffer search with 3 against 6 candidates per buffer
l() {
  for i in 1 2; do
    timeout -k 10 200 tools/place_buffers 4096 3 3 5 6 >> gpurun_out/r05l_m3.jsonl 2>&1 &&
    timeout -k 10 300 tools/place_buffers 4096 6 3 5 6 >> gpurun_out/r05l_m6.jsonl 2>&1 || return 1
  done
}

# m: the product probe with repeated sweeps over 10 contexts; its tests; the bench three times
m() {
  timeout -k 10 300 python -u tools/probe_trials.py --n 10 --hold 5 > gpurun_out/r05m_trials.jsonl 2>&1 &&
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cg_paths_gpu.py \
    -k placement > gpurun_out/r05m_tests.log 2>&1 || return 1
  for i in 1 2 3; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r05m_bench.jsonl 2>> gpurun_out/r05m_bench.err || return 1
  done
}

# o: loopback kernel timelines at 4096x1024 and 4096x2048
o() {
  rm -rf gpurun_out/r05o_*
  for s in 4096x1024 4096x2048; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05o_$s -o run -- python -u \
      tools/loopback_probe.py --shapes $s --iters 60 --rounds 1 --applies 10 > gpurun_out/r05o_$s.log 2>&1 || return 1
  done
}

# p: t-shard edge launch chunk length on the loopback (edge_xchunk)
p() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5"
  for r in 1 2; do
    for e in 16 8 12 4; do
      SM_TEST_OPTS=edge_xchunk=$e timeout -k 10 300 $L > gpurun_out/r05p_e${e}_$r.log 2>&1 || return 1
    done
  done
}

# q: longer edge chunks (interior + edge tiles within one dispatch round at 4096x1024)
q() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5"
  for r in 1 2; do
    for e in 16 32 24; do
      SM_TEST_OPTS=edge_xchunk=$e timeout -k 10 300 $L > gpurun_out/r05q_e${e}_$r.log 2>&1 || return 1
    done
  done
}

# r: the edge-chunk residency rule on the loopback (default) against fixed 16, and the t-shard tests
r() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5"
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py \
    tests/test_cg_paths_gpu.py -k "tshard or loop or shard" > gpurun_out/r05r_tests.log 2>&1 || return 1
  for i in 1 2; do
    timeout -k 10 300 $L > gpurun_out/r05r_rule_$i.log 2>&1 &&
    SM_TEST_OPTS=edge_xchunk=16 timeout -k 10 300 $L > gpurun_out/r05r_e16_$i.log 2>&1 || return 1
  done
}

# s: the t-shard apply without its edge columns (apply_split=2) -- bitwise tests, then the
#    loopback's apply time per schedule, twice
s() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 100 --rounds 2 --applies 20"
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    -k apply_modes > gpurun_out/r05s_tests.log 2>&1 || return 1
  for i in 1 2; do
    for m in 0 1 2; do
      SM_TEST_OPTS=apply_split=$m timeout -k 10 300 $L > gpurun_out/r05s_split${m}_$i.log 2>&1 || return 1
    done
  done
}

# u: where the CG pass's extra reads come from -- L2 counters and timing per launch geometry
#    (waves per block, rows per block) at 4096^2 with the link codes
u() {
  rm -rf gpurun_out/r05u_*
  for g in 1,64 1,128 1,32 2,64 4,64 2,32; do
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
      -d gpurun_out/r05u_pmc_${g/,/_} -o run -- python3 tools/tune_shapes.py 4096x4096:$g,1 --iters 30 --rounds 1 \
      > gpurun_out/r05u_pmc_${g/,/_}.log 2>&1 || return 1
  done
  timeout -k 10 300 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:1,128,1 4096x4096:1,32,1 \
    4096x4096:2,64,1 4096x4096:4,64,1 4096x4096:2,32,1 --iters 100 --rounds 3 > gpurun_out/r05u_time.log 2>&1
}

# w: read request sizes (32 / 64 / 128 B) of the CG pass and the apply
w() {
  rm -rf gpurun_out/r05w_*
  local P="python3 bench.py --steps 10 --warmup 2 --applies 4 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    --output-format csv -d gpurun_out/r05w_sizes -o run -- $P > gpurun_out/r05w_sizes.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc TCC_REQ_sum TCC_READ_sum TCC_STREAMING_REQ_sum TCC_BUBBLE_sum \
    --output-format csv -d gpurun_out/r05w_req -o run -- $P > gpurun_out/r05w_req.log 2>&1
}

# x: read requests of the CG pass when the halo lanes of the named streams load owned columns
#    (counter-only variants, tools/exp_halo_build.py; wrong values, traffic only)
x() {
  rm -rf gpurun_out/r05x_*
  local T="python3 tools/tune_shapes.py 4096x4096:1,64,1 --iters 30 --rounds 1"
  for v in base d1 d2 uc x all; do
    local lib=""
    [ $v != base ] && lib=$PWD/tools/exp/libsm_hip_$v.so
    SM_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_READ_sum \
      --output-format csv -d gpurun_out/r05x_$v -o run -- $T > gpurun_out/r05x_$v.log 2>&1 || return 1
  done
}

# z: A/B of the product library against tools/ab_libs/libsm_hip_base.so (the previous build), ABAB x4,
#    the driver's bench at 200 steps without the extras; then the CG parity subset on the product
z() {
  local B="python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  for i in 1 2 3 4; do
    SM_LIB_PATH=$PWD/tools/ab_libs/libsm_hip_base.so SM_LIB_AB=1 timeout -k 10 200 $B > gpurun_out/r05z_base_$i.log 2>&1 &&
    timeout -k 10 200 $B > gpurun_out/r05z_new_$i.log 2>&1 || return 1
  done
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_cg_paths_gpu.py \
    -k "cg" > gpurun_out/r05z_tests.log 2>&1
}

# ab: the apply with odd x-chunks marching backward -- bitwise tests, apply time A/B (apply_alt=0 / 1, x4),
#     L2 read counters per variant
ab() {
  rm -rf gpurun_out/r05ab_*
  timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_large.py -k "march_directions or operators_bitwise or oracle_parity or large_lattice" \
    > gpurun_out/r05ab_tests.log 2>&1 || return 1
  local B="python3 bench.py --steps 20 --warmup 5 --applies 200 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  for i in 1 2 3 4; do
    SM_TEST_OPTS=apply_alt=0 timeout -k 10 200 $B > gpurun_out/r05ab_fwd_$i.log 2>&1 &&
    timeout -k 10 200 $B > gpurun_out/r05ab_alt_$i.log 2>&1 || return 1
  done
  local P="python3 bench.py --steps 4 --warmup 2 --applies 10 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  SM_TEST_OPTS=apply_alt=0 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
    -d gpurun_out/r05ab_pmc_fwd -o run -- $P > gpurun_out/r05ab_pmc_fwd.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
    -d gpurun_out/r05ab_pmc_alt -o run -- $P > gpurun_out/r05ab_pmc_alt.log 2>&1
}

# ac: apply variants 1 (all forward) and 3 (odd x-chunks backward) interleaved in ONE process on the same
#     buffers, 32 / 64-row chunks, D and D^dag, twice
ac() {
  for d in 0 1 0 1; do
    timeout -k 10 300 python3 -u tools/tune_dslash.py --bt 256 --xchunk 32,64 --remap 1 --variant 1,3 --rounds 15 \
      --applies 50 --dagger $d >> gpurun_out/r05ac_d$d.jsonl 2>&1 || return 1
  done
}

# ad: the N > 1 bench path rehearsed on one GPU with host-staged halos (4 and 8 ranks: spawn, barrier,
#     max over ranks, one JSON line)
ad() {
  timeout -k 10 400 python3 bench.py --gpus 4 --transport hosted --steps 20 --warmup 5 > gpurun_out/r05ad_bench4.log 2>&1 &&
  timeout -k 10 500 python3 bench.py --gpus 8 --transport hosted --steps 20 --warmup 5 > gpurun_out/r05ad_bench8.log 2>&1
}

# ae: 4096 x 512 shards (config 4 over 8 GPUs, the weak slab): rows per block, one-wave blocks, codes on
ae() {
  timeout -k 10 300 python3 -u tools/tune_shapes.py 4096x512:1,48,1 4096x512:1,40,1 4096x512:1,32,1 4096x512:1,24,1 \
    4096x512:1,21,1 4096x512:1,20,1 4096x512:1,16,1 4096x512:1,64,1 4096x512:1,48,0 --iters 200 --rounds 5 \
    > gpurun_out/r05ae_4096x512.log 2>&1 &&
  timeout -k 10 300 python3 -u tools/tune_shapes.py 4096x1024:1,40,1 4096x1024:1,32,1 4096x1024:1,21,1 4096x1024:1,64,1 \
    4096x2048:1,32,1 4096x2048:1,40,1 4096x2048:1,64,1 --iters 100 --rounds 5 >> gpurun_out/r05ae_4096x512.log 2>&1
}

# af: 4096 x 512 rows per block (one dispatch round: 21) in the plain shard and through the loopback
af() {
  timeout -k 10 300 python3 -u tools/tune_shapes.py 4096x512:1,48,0 4096x512:1,21,0 4096x512:1,24,0 4096x512:1,22,0 \
    4096x512:1,25,0 4096x512:1,21,1 --iters 200 --rounds 5 > gpurun_out/r05af_shapes.log 2>&1 || return 1
  for i in 1 2; do
    for g in 1,48 1,21 1,24; do
      timeout -k 10 200 python -u tools/loopback_probe.py --shapes 4096x512 --iters 200 --rounds 3 --applies 5 --geom $g \
        >> gpurun_out/r05af_loopback.log 2>&1 || return 1
    done
  done
}

# fin: the round-end evidence set after the gate (tag $1): benches, config 5, rocprof stats + step
#      gap, FETCH / WRITE passes, the loopback, and the placement probe over 10 contexts
fin() {
  local T=${1:-cur}
  rm -rf gpurun_out/prof_stats_$T gpurun_out/prof_fetch_$T gpurun_out/prof_write_$T
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/build_id_$T.txt &&
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$T.log 2>&1 &&
  timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 &&
  timeout -k 10 300 python3 bench.py --gpus 2 --transport hosted --steps 50 --warmup 10 --no-weak > gpurun_out/bench2_$T.log 2>&1 &&
  timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench_c5_$T.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats_$T -o run -- python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak --evolved-trajectories 0 > gpurun_out/prof_stats_$T.log 2>&1 &&
  python3 tools/step_gap.py gpurun_out/prof_stats_$T/run_kernel_trace.csv --last 200 > gpurun_out/step_gap_$T.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline --no-weak --evolved-trajectories 0 > gpurun_out/prof_fetch_$T.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$T -o run -- python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline --no-weak --evolved-trajectories 0 > gpurun_out/prof_write_$T.log 2>&1 &&
  timeout -k 10 300 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048,4096x4096 --iters 100 --rounds 2 > gpurun_out/loopback_$T.log 2>&1 &&
  timeout -k 10 300 python -u tools/probe_trials.py --n 10 --hold 5 > gpurun_out/probe_trials_$T.jsonl 2>&1
}

# gate: the full GPU gate in natural order, then smoke (tag $2)
gate() {
  local T=${1:-cur}
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/build_id_$T.txt &&
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gate_$T.log 2>&1 &&
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
}

"$@"
