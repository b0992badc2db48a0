# Round 3: the KFD queue / scheduler properties of the box (stall diagnosis),
# then the full GPU gate in natural order with the current build. Tag $1.
export TMPDIR=/tmp
T=${1:-cur}
mkdir -p gpurun_out
( for f in /sys/class/kfd/kfd/topology/nodes/*/properties; do echo "== $f"; grep -E "simd_count|max_waves|cu_per_simd|num_cp_queues|num_sdma|num_xcc|max_slots|gfx_target|vendor_id|device_id|array_count|simd_per_cu|mem_banks|caches" $f; done; cat /sys/module/amdgpu/parameters/hws_max_conc_proc /sys/module/amdgpu/parameters/sched_policy /sys/module/amdgpu/parameters/max_num_of_queues_per_device /sys/module/amdgpu/parameters/vm_update_mode 2>&1; echo "GPU_MAX_HW_QUEUES=$GPU_MAX_HW_QUEUES" ) > gpurun_out/kfd_props_$T.txt 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/gputests_$T.log 2>&1
