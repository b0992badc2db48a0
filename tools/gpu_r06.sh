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

# c: the RCCL total order (one communicator, events between the two streams) against round 5 on the
#    loopback, twice; the RCCL / t-shard tests; the link-offset drift histogram at config 3
c() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 20"
  for i in 1 2; do
    timeout -k 10 300 $L > gpurun_out/r06c_order_$i.log 2>&1 &&
    SM_LIB_PATH=$PWD/tools/ab_libs/libsm_hip_r05.so SM_LIB_AB=1 timeout -k 10 300 $L > gpurun_out/r06c_r05_$i.log 2>&1 || return 1
  done
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    tests/test_dist_gpu.py tests/test_gpu_parity.py -k "loopback or sharded or link" \
    > gpurun_out/r06c_tests.log 2>&1 &&
  timeout -k 10 300 python -u tools/link_drift.py --at 0,50,500,2000 > gpurun_out/r06c_drift.jsonl 2>&1
}

# d: the t-strip CG pass -- its tests, then the strip against the window pass at 4096^2 (one process,
#    interleaved; chunk lengths for whole dispatch rounds), and the loopback / drift runs of c
d() {
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cg_strip_gpu.py \
    > gpurun_out/r06d_tests.log 2>&1 &&
  timeout -k 10 400 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:4,64,1,1,0 4096x4096:4,69,1,1,1 \
    4096x4096:4,32,1,1,0 4096x4096:4,128,1,1,0 4096x4096:4,137,1,1,1 --iters 100 --rounds 4 > gpurun_out/r06d_shapes.log 2>&1 &&
  c
}

# e: RCCL ordering events on / off on the loopback; t-strip shapes (4 and 2 waves) at 4096^2 and their
#    L2 / SQ counters against the window pass
e() {
  rm -rf gpurun_out/r06e_*
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 3 --applies 5"
  for i in 1 2; do
    timeout -k 10 300 $L > gpurun_out/r06e_order_$i.log 2>&1 &&
    SM_TEST_OPTS=rccl_order=0 timeout -k 10 300 $L > gpurun_out/r06e_noorder_$i.log 2>&1 || return 1
  done
  timeout -k 10 400 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:4,69,1,1,1 4096x4096:2,71,1,1,1 \
    4096x4096:2,141,1,1,1 4096x4096:2,32,1,1,0 4096x4096:4,69,1,1,0 --iters 100 --rounds 4 > gpurun_out/r06e_shapes.log 2>&1 || return 1
  for g in 1,64,1 4,69,1,1,1 2,71,1,1,1; do
    local t=${g//,/_}
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
      -d gpurun_out/r06e_tcc_$t -o run -- python3 tools/tune_shapes.py 4096x4096:$g --iters 30 --rounds 1 \
      > gpurun_out/r06e_tcc_$t.log 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
      SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r06e_sq_$t -o run -- \
      python3 tools/tune_shapes.py 4096x4096:$g --iters 30 --rounds 1 > gpurun_out/r06e_sq_$t.log 2>&1 || return 1
  done
}

# f: chunk alignment (power-of-two vs balanced chunks) for the window and strip passes at 4096^2;
#    the t-shard edge rows per block under the RCCL ordering events on the loopback
f() {
  timeout -k 10 500 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:1,69,1,0,1 4096x4096:4,69,1,1,1 \
    4096x4096:4,64,1,1,0 4096x4096:2,64,1,1,0 4096x4096:4,32,1,1,0 4096x4096:1,32,1 4096x4096:1,128,1 \
    --iters 100 --rounds 4 > gpurun_out/r06f_shapes.log 2>&1 || return 1
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 3 --applies 5"
  for e in 16 8 12 24; do
    SM_TEST_OPTS=edge_xchunk=$e timeout -k 10 300 $L > gpurun_out/r06f_edge$e.log 2>&1 || return 1
  done
}

# g: t-shard face schedules on the loopback (pipelined behind the edge launch with ordering events, the same
#    without them, deferred to the next pass), and their tests
g() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5"
  for i in 1 2; do
    SM_TEST_OPTS=face_pipe=1 timeout -k 10 300 $L > gpurun_out/r06g_pipe1_$i.log 2>&1 &&
    SM_TEST_OPTS=face_pipe=2 timeout -k 10 300 $L > gpurun_out/r06g_pipe2_$i.log 2>&1 &&
    SM_TEST_OPTS=face_pipe=1,rccl_order=0 timeout -k 10 300 $L > gpurun_out/r06g_pipe1_noorder_$i.log 2>&1 || return 1
  done
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cg_paths_gpu.py \
    tests/test_rccl_loopback_gpu.py -k "tshard or loopback" > gpurun_out/r06g_tests.log 2>&1
}

# h: the full GPU gate and smoke, then the driver's bench command twice and the 200-step default
#    (probe kept time against the sustained pass)
h() {
  gate h &&
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06h_bench_driver1.log 2>&1 &&
  timeout -k 10 400 python3 bench.py > gpurun_out/r06h_bench200.log 2>&1 &&
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06h_bench_driver2.log 2>&1
}

# i: the placement probe on drawn data -- its tests, ten contexts in one process, the driver's bench command
#    three times (probe kept time against the sustained pass)
i() {
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cg_paths_gpu.py \
    -k placement > gpurun_out/r06i_tests.log 2>&1 &&
  timeout -k 10 300 python -u tools/probe_trials.py --n 10 --hold 5 > gpurun_out/r06i_trials.jsonl 2>&1 || return 1
  for k in 1 2 3; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/r06i_bench.jsonl 2>> gpurun_out/r06i_bench.err || return 1
  done
}

# j: device-initiated transport feasibility (tools/peer_probe: one process against itself, two processes
#    on one GPU over IPC-opened uncached / coarse regions), then RCCL launch settings on the loopback
j() {
  local P="timeout -k 5 90 tools/peer_probe"
  $P loop 2000 8192 1 > gpurun_out/r06j_peer.jsonl 2>&1 &&
  $P ipc 2000 8192 1 >> gpurun_out/r06j_peer.jsonl 2>&1 &&
  $P ipc 2000 8192 0 >> gpurun_out/r06j_peer.jsonl 2>&1 &&
  $P ipc 2000 16 1 >> gpurun_out/r06j_peer.jsonl 2>&1 || return 1
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024 --iters 200 --rounds 2 --applies 20"
  timeout -k 10 300 $L > gpurun_out/r06j_default.log 2>&1 &&
  NCCL_GRAPH_MIXING_SUPPORT=0 timeout -k 10 300 $L > gpurun_out/r06j_nomix.log 2>&1 &&
  NCCL_LAUNCH_MODE=GROUP timeout -k 10 300 $L > gpurun_out/r06j_group.log 2>&1
}

# k: the peer transport -- its tests (loopback and 2-8 processes on the one GPU), then the loopback probe
#    with the plain shard, the RCCL loopback and the peer loopback side by side
k() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_peer_gpu.py \
    > gpurun_out/r06k_tests.log 2>&1 &&
  timeout -k 10 400 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 \
    --applies 20 > gpurun_out/r06k_loopback.log 2>&1
}

# l: bench with the peer transport rehearsed on one GPU (2 and 4 ranks sharing it: the check against the
#    host-staged transport, the path, not a scaling figure), the one-GPU bench, and the RCCL / hosted tests
l() {
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06l_bench1.log 2>&1 &&
  timeout -k 10 400 python3 bench.py --gpus 2 --device 0 --steps 50 --warmup 10 --no-cpu-baseline \
    > gpurun_out/r06l_bench2_peer.log 2>&1 &&
  timeout -k 10 400 python3 bench.py --gpus 4 --device 0 --steps 50 --warmup 10 --no-cpu-baseline --no-weak \
    > gpurun_out/r06l_bench4_peer.log 2>&1 &&
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    tests/test_dist_gpu.py -k "loopback_equals or sharded_gpu_path or recompute" > gpurun_out/r06l_tests.log 2>&1
}

# m: peer faces staged in LDS and written out coalesced -- the peer tests, the loopback probe, and the
#    one-GPU bench against the library before the peer transport (tools/ab_libs/libsm_hip_pre_peer.so), ABAB
m() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_peer_gpu.py \
    > gpurun_out/r06m_tests.log 2>&1 &&
  timeout -k 10 400 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 \
    --applies 20 > gpurun_out/r06m_loopback.log 2>&1 || return 1
  local B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --evolved-trajectories 0"
  for i in 1 2; do
    timeout -k 10 300 $B >> gpurun_out/r06m_ab_new.jsonl 2>> gpurun_out/r06m_ab.err &&
    SM_LIB_PATH=$PWD/tools/ab_libs/libsm_hip_pre_peer.so SM_LIB_AB=1 timeout -k 10 300 $B \
      >> gpurun_out/r06m_ab_old.jsonl 2>> gpurun_out/r06m_ab.err || return 1
  done
}

# n: the peer tests and the loopback probe (plain / RCCL / peer) on the current build
n() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_peer_gpu.py \
    > gpurun_out/r06n_tests.log 2>&1 &&
  timeout -k 10 400 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 \
    --applies 20 > gpurun_out/r06n_loopback.log 2>&1
}

# o: the peer pass's face-store forms A/B on the peer loopback (16-B write-through, 8-B atomic, plain), twice
o() {
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5 --contexts one,peer"
  for i in 1 2; do
    for m in 0 1 2; do
      SM_TEST_OPTS=peer_store=$m timeout -k 10 300 $L > gpurun_out/r06o_store${m}_$i.log 2>&1 || return 1
    done
  done
  SM_TEST_OPTS=peer_store=2 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_peer_gpu.py > gpurun_out/r06o_tests_plain.log 2>&1
}

# p: the peer pass with the shape's march schedule -- peer tests, the loopback probe, then the full gate
p() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_peer_gpu.py \
    > gpurun_out/r06p_tests.log 2>&1 &&
  timeout -k 10 400 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 \
    --applies 5 --contexts one,peer > gpurun_out/r06p_loopback.log 2>&1 &&
  gate p
}

# q: configs 4 and 5 at full size over the peer transport (8 processes on the one GPU)
q() {
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_configs_gpu.py \
    -k "sharded and peer" > gpurun_out/r06q_tests.log 2>&1
}

# r: the drop-in shim's tests (the peer transport through MPI_Allgather included) and the 2-rank peer bench
#    rehearsal with the timed-solve residual check
r() {
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dropin_gpu.py \
    > gpurun_out/r06r_tests.log 2>&1 &&
  timeout -k 10 300 python3 bench.py --gpus 2 --device 0 --steps 50 --warmup 10 --no-weak --no-cpu-baseline \
    > gpurun_out/r06r_bench2.log 2>&1
}

# s: the HMC program as 2 MPI ranks over the peer transport (conf gather through shard 0's mailbox)
s() {
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hmc_gpu.py \
    -k "program" > gpurun_out/r06s_tests.log 2>&1
}

# t: the N > 1 bench paths rehearsed on one GPU: the host-staged headline with the peer transport timed beside it
#    (the code path of the RCCL default), 2 and 4 ranks; the peer headline, 2 ranks
t() {
  timeout -k 10 400 python3 bench.py --gpus 2 --device 0 --transport hosted --steps 50 --warmup 10 --no-weak \
    --no-cpu-baseline > gpurun_out/r06t_bench2_hosted.log 2>&1 &&
  GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python3 bench.py --gpus 4 --device 0 --transport hosted --steps 50 --warmup 10 \
    --no-weak --no-cpu-baseline > gpurun_out/r06t_bench4_hosted.log 2>&1 &&
  timeout -k 10 400 python3 bench.py --gpus 2 --device 0 --transport peer --steps 50 --warmup 10 --no-weak \
    --no-cpu-baseline > gpurun_out/r06t_bench2_peer.log 2>&1
}

# u: RCCL contexts with the CG sums all-reduced in the pass (peer headers) -- the RCCL loopback tests, then
#    the loopback probe against rccl_sums=1 (ncclAllReduce per pass), twice
u() {
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    tests/test_cg_paths_gpu.py -k "loopback or tshard" > gpurun_out/r06u_tests.log 2>&1 || return 1
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5 --contexts one,loopback"
  for i in 1 2; do
    timeout -k 10 300 $L > gpurun_out/r06u_psums_$i.log 2>&1 &&
    SM_TEST_OPTS=rccl_sums=1 timeout -k 10 300 $L > gpurun_out/r06u_ncclsums_$i.log 2>&1 || return 1
  done
}

# v: the in-pass sums over split launches with several shards (hosted_psums), then the peer tests, RCCL loopback
v() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_peer_gpu.py \
    tests/test_rccl_loopback_gpu.py > gpurun_out/r06v_tests.log 2>&1 &&
  timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_dist_gpu.py \
    -k "sharded_gpu_path" > gpurun_out/r06v_tests2.log 2>&1
}

# w: kernel-trace timelines of the t-shard CG pass at 4096 x 512 through the RCCL loopback (split launches, the
#    face exchange, in-pass sums) and the peer loopback (one launch)
w() {
  local L="python3 -u tools/loopback_probe.py --shapes 4096x512 --iters 60 --rounds 1 --applies 1 --warmup 5"
  for ctx in loopback peer; do
    rm -rf gpurun_out/r06w_$ctx
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06w_$ctx -o run -- $L --contexts $ctx \
      > gpurun_out/r06w_$ctx.log 2>&1 &&
    python3 tools/trace_pass.py gpurun_out/r06w_$ctx/run_kernel_trace.csv --last 40 > gpurun_out/r06w_${ctx}_trace.txt 2>&1 \
      || return 1
  done
}

# x: the stream-ordering events without / with the system-scope fence on the RCCL loopback (twice each), the
#    RCCL loopback tests, then the traces of w (ran on a build with test option ev_fence, since reverted: no effect)
x() {
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    > gpurun_out/r06x_tests.log 2>&1 || return 1
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 20 --contexts one,loopback"
  for i in 1 2; do
    timeout -k 10 300 $L > gpurun_out/r06x_nofence_$i.log 2>&1 &&
    SM_TEST_OPTS=ev_fence=1 timeout -k 10 300 $L > gpurun_out/r06x_fence_$i.log 2>&1 || return 1
  done
  w
}

# y: the link codes stored per site (code_ilv=1) against the two planes -- its tests and the link tests with
#    the option on, four interleaved bench pairs (200 steps), then the pass's L2 counters both ways (ran on build
#    17ede56d9968562b with test option code_ilv, since removed: reads unchanged, 0.4 % slower)
y() {
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/r06y_build_id.txt &&
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "link" > gpurun_out/r06y_tests.log 2>&1 &&
  SM_TEST_OPTS=code_ilv=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_cg_paths_gpu.py -k "link or cg_vs_reference or tshard" \
    > gpurun_out/r06y_tests_ilv.log 2>&1 || return 1
  local B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  for i in 1 2 3 4; do
    SM_TEST_OPTS=code_ilv=1 timeout -k 10 300 $B > gpurun_out/r06y_ilv_$i.log 2>&1 &&
    timeout -k 10 300 $B > gpurun_out/r06y_planes_$i.log 2>&1 || return 1
  done
  for m in 0 1; do
    SM_TEST_OPTS=code_ilv=$m timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
      --output-format csv -d gpurun_out/r06y_tcc_$m -o run -- python3 tools/tune_shapes.py 4096x4096:1,64,1 \
      --iters 30 --rounds 1 > gpurun_out/r06y_tcc_$m.log 2>&1 || return 1
  done
}

# z: the t-shard CG pass's stream hand-offs on events recorded by the launches themselves (kernel_events=1,
#    the new default) against markers (0): the RCCL loopback and in-pass-sums tests, the loopback twice each way
z() {
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/r06z_build_id.txt &&
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    tests/test_cg_paths_gpu.py tests/test_peer_gpu.py -k "loopback or tshard or in_pass" > gpurun_out/r06z_tests.log 2>&1 || return 1
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5 --contexts one,loopback"
  for i in 1 2; do
    timeout -k 10 300 $L > gpurun_out/r06z_kev1_$i.log 2>&1 &&
    SM_TEST_OPTS=kernel_events=0 timeout -k 10 300 $L > gpurun_out/r06z_kev0_$i.log 2>&1 || return 1
  done
}

# aa: the RCCL / host-staged t-shard CG pass as one launch (test option rccl_onelaunch, since removed: faces
#     exchanged behind the pass on the comm stream, the next pass's face-reading waves waiting for a flag) -- the
#     RCCL loopback, t-shard schedule and in-pass-sums tests, then the loopback against the split launches, twice.
#     Ran on builds 6bdcb069660ca470 (slower) and 920ae3ae89b8fbc1 (a wait timed out: DESIGN §7)
aa() {
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/r06aa_build_id.txt &&
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_loopback_gpu.py \
    tests/test_cg_paths_gpu.py tests/test_peer_gpu.py tests/test_dist_gpu.py -k "loopback or tshard or in_pass or sharded" \
    > gpurun_out/r06aa_tests.log 2>&1 || return 1
  local L="python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048 --iters 200 --rounds 3 --applies 5 --contexts one,loopback,peer"
  for i in 1 2; do
    timeout -k 10 300 $L > gpurun_out/r06aa_one_$i.log 2>&1 &&
    SM_TEST_OPTS=rccl_onelaunch=0 timeout -k 10 300 $L > gpurun_out/r06aa_split_$i.log 2>&1 || return 1
  done
}

# ab: (build 7947ebe3c99e0868 + tools/exp_stream_build.py) where the CG pass's reads above its algorithmic bytes go -- the pass's L2 read requests with each stream
#     pinned to one row per tile (counter-only libraries from tools/exp_stream_build.py; wrong values) against
#     the product library, 4096^2; then the x-halo rows alone (d1h, d2h, uh, allh)
ab() {
  for v in ${AB_VARIANTS:-base d1 d2 u x d1h d2h uh allh}; do
    (
      if [ "$v" != base ]; then export SM_LIB_PATH=$PWD/tools/exp/libsm_hip_s_$v.so; fi
      timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
        -d gpurun_out/r06ab_tcc_$v -o run -- python3 tools/tune_shapes.py 4096x4096:1,64,1 --iters 30 --rounds 1 \
        > gpurun_out/r06ab_tcc_$v.log 2>&1
    ) || return 1
  done
}

# ac: 2-wave blocks on x-adjacent chunks of one t-window (test option ra_xpair=1, since removed: slower, more
#     reads; ran on build 45632ff9269128ae) at 4096^2 -- its tests, four interleaved bench pairs (200 steps), then
#     the pass's L2 read requests both ways
ac() {
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cg_paths_gpu.py \
    -k "xpair or ticketed" > gpurun_out/r06ac_tests.log 2>&1 || return 1
  local B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  for i in 1 2 3 4; do
    SM_TEST_OPTS=ra_xpair=1 timeout -k 10 300 $B > gpurun_out/r06ac_xpair_$i.log 2>&1 &&
    timeout -k 10 300 $B > gpurun_out/r06ac_default_$i.log 2>&1 || return 1
  done
  for m in 0 1; do
    SM_TEST_OPTS=ra_xpair=$m timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
      --output-format csv -d gpurun_out/r06ac_tcc_$m -o run -- python3 bench.py --steps 30 --warmup 5 --applies 5 \
      --no-cpu-baseline --no-weak --evolved-trajectories 0 > gpurun_out/r06ac_tcc_$m.log 2>&1 || return 1
  done
}

# ad: one dispatch round of long chunks at 4096^2 (27 x 152 / 26 x 160 rows: 1998 / 1924 one-wave tiles for
#     2048 slots; the x-halo rows are 5 % of a chunk instead of 12.5 %) against 64 / 128-row chunks, interleaved
ad() {
  timeout -k 10 400 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:1,152,1 4096x4096:1,160,1 \
    4096x4096:1,152,1,0,1 4096x4096:1,128,1 4096x4096:1,256,1 --iters 100 --rounds 4 > gpurun_out/r06ad_shapes.log 2>&1
}

# ae: whole dispatch rounds at 4096^2 (74 wave columns x balanced chunks: 55 chunks = 4070 tiles ~ 2 rounds of 2048,
#     52 = 3848, 40 = 2960, 27 = 1998) against the default 64-row chunks, interleaved
ae() {
  timeout -k 10 500 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:1,75,1,0,1 4096x4096:1,76,1 \
    4096x4096:1,79,1,0,1 4096x4096:1,103,1,0,1 4096x4096:1,152,1 --iters 100 --rounds 5 > gpurun_out/r06ae_shapes.log 2>&1
}

# af: balanced chunk counts 34..48 at 4096^2 (the 40-chunk form won in ae) against the default, interleaved
af() {
  timeout -k 10 600 python3 -u tools/tune_shapes.py 4096x4096:1,64,1 4096x4096:1,121,1,0,1 4096x4096:1,114,1,0,1 \
    4096x4096:1,108,1,0,1 4096x4096:1,103,1,0,1 4096x4096:1,98,1,0,1 4096x4096:1,94,1,0,1 4096x4096:1,90,1,0,1 \
    4096x4096:1,86,1,0,1 --iters 100 --rounds 5 > gpurun_out/r06af_shapes.log 2>&1
}

# ag: 40 balanced chunks (102-103 rows) at 4096^2 as the context's geometry from creation (the placement probe
#     then tunes for it: SM_TEST_OPTS ra_xchunk=103,ra_xbal=1) against the default, four interleaved bench pairs
ag() {
  local B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  for i in 1 2 3 4; do
    SM_TEST_OPTS=ra_xchunk=103,ra_xbal=1 timeout -k 10 300 $B > gpurun_out/r06ag_c40_$i.log 2>&1 &&
    timeout -k 10 300 $B > gpurun_out/r06ag_default_$i.log 2>&1 || return 1
  done
}

# ah: the Dirac apply's rows per block at 4096^2 (bt 256, XCD map, two-row lookahead), interleaved -- the CG pass's
#     chunk count had one sharp optimum (af)
ah() {
  timeout -k 10 400 python3 -u tools/tune_dslash.py --bt 256 --xchunk 24,26,28,30,32,34,36,40,43,48,52,64 --remap 1 \
    --variant 1 --rounds 5 --applies 20 > gpurun_out/r06ah_apply_rows.log 2>&1
}

# ai: rows per block of the t-shard CG pass at 4096 x 512 (config 4's 8-GPU shard): one shard and the RCCL loopback
ai() {
  for x in 48 32 40 56 64 73 86 103 128; do
    timeout -k 10 200 python -u tools/loopback_probe.py --shapes 4096x512 --iters 200 --rounds 3 --applies 2 \
      --contexts one,loopback --geom 1,$x > gpurun_out/r06ai_rows_$x.log 2>&1 || return 1
  done
}

# aj: the t-shard pass at 4096 x 512 around 32 rows per block, twice, interleaved (RCCL loopback and one shard)
aj() {
  for i in 1 2; do
    for x in 48 24 28 32 36; do
      timeout -k 10 200 python -u tools/loopback_probe.py --shapes 4096x512 --iters 200 --rounds 3 --applies 2 \
        --contexts one,loopback --geom 1,$x > gpurun_out/r06aj_rows_${x}_$i.log 2>&1 || return 1
    done
  done
}

# ak: rows per block of the t-shard CG pass at 4096 x 1024 and 4096 x 2048 (4 and 2 GPUs), RCCL loopback and one shard
ak() {
  for x in 40 28 32 48; do
    timeout -k 10 200 python -u tools/loopback_probe.py --shapes 4096x1024 --iters 200 --rounds 3 --applies 2 \
      --contexts one,loopback --geom 1,$x > gpurun_out/r06ak_1024_rows_$x.log 2>&1 || return 1
  done
  for x in 32 24 28 40; do
    timeout -k 10 200 python -u tools/loopback_probe.py --shapes 4096x2048 --iters 100 --rounds 3 --applies 2 \
      --contexts one,loopback --geom 1,$x > gpurun_out/r06ak_2048_rows_$x.log 2>&1 || return 1
  done
}

# al: balanced chunk counts of the 8192^2 pass (config 5; 4-wave blocks, 37 t-blocks) against its 32-row chunks
al() {
  timeout -k 10 600 python3 -u tools/tune_shapes.py 8192x8192:4,32,1 8192x8192:4,35,1,0,1 8192x8192:4,41,1,0,1 \
    8192x8192:4,52,1,0,1 8192x8192:4,64,1 8192x8192:4,103,1,0,1 8192x8192:1,64,1 --iters 30 --rounds 3 \
    > gpurun_out/r06al_shapes_8192.log 2>&1
}

# fin: the round-end evidence set after the gate (tag $1): benches, config 5, rocprof stats + step gap, FETCH / WRITE
#      passes, the loopback, and the placement probe over 10 contexts
fin() {
  local T=${1:-cur}
  rm -rf gpurun_out/prof_stats_$T gpurun_out/prof_fetch_$T gpurun_out/prof_write_$T
  local P="python3 bench.py --steps 10 --warmup 2 --applies 10 --no-cpu-baseline --no-weak --evolved-trajectories 0"
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/build_id_$T.txt &&
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_$T.log 2>&1 &&
  timeout -k 10 400 python3 bench.py > gpurun_out/bench_$T.log 2>&1 &&
  timeout -k 10 300 python3 bench.py --gpus 2 --device 0 --transport hosted --steps 50 --warmup 10 --no-weak \
    > gpurun_out/bench2_$T.log 2>&1 &&
  GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python3 bench.py --gpus 8 --device 0 --transport peer --steps 50 --warmup 10 \
    --no-weak --no-cpu-baseline > gpurun_out/bench8_$T.log 2>&1 &&
  timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench_c5_$T.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats_$T -o run -- python3 bench.py --steps 200 --warmup 20 --applies 20 --no-cpu-baseline --no-weak --evolved-trajectories 0 > gpurun_out/prof_stats_$T.log 2>&1 &&
  python3 tools/step_gap.py gpurun_out/prof_stats_$T/run_kernel_trace.csv --last 200 > gpurun_out/step_gap_$T.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$T -o run -- $P > gpurun_out/prof_fetch_$T.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$T -o run -- $P > gpurun_out/prof_write_$T.log 2>&1 &&
  timeout -k 10 400 python -u tools/loopback_probe.py --shapes 4096x512,4096x1024,4096x2048,4096x4096 --iters 100 --rounds 2 \
    --contexts one,loopback,peer > gpurun_out/loopback_$T.log 2>&1 &&
  timeout -k 10 300 python -u tools/probe_trials.py --n 10 --hold 5 > gpurun_out/probe_trials_$T.jsonl 2>&1
}

# gate: the full GPU gate in natural order, then smoke (tag $1)
gate() {
  local T=${1:-cur}
  python3 -c "import schwingermodel_amd as s; print(s.lib.sm_build_id().decode())" > gpurun_out/build_id_$T.txt &&
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gate_$T.log 2>&1 &&
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
}

"$@"
