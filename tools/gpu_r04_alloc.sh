# Round 4: why the CG pass runs faster on fields in
# allocations of >= 2 GiB than on own-size (512 MiB) allocations at 4096^2.
# tools/stride_probe runs the product launcher on 5 streamed fields, each in
# its own allocation of 2V (own size) or 8V (2 GiB) double2. First the pass
# time, interleaved; then address-translation (UTCL1), L2 / fabric and UTCL2
# counters, one rocprofv3 --pmc pass per counter group. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 100 tools/stride_probe 4096x4096 1,2,0,1,2 1,2,0,1,8 >> gpurun_out/alloc_time_$T.jsonl 2>&1 || exit 1
done
i=0
for pm in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
          "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum" \
          "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum"; do
  i=$((i+1))
  for lay in 1,2,0,1,2 1,2,0,1,8; do
    d=gpurun_out/alloc_pmc${i}_${lay//,/_}_$T
    rm -rf $d
    timeout -s KILL 120 rocprofv3 --pmc $pm --output-format csv -d $d -o run -- tools/stride_probe 4096x4096 $lay > $d.log 2>&1 || exit 1
  done
done
