# Submit ONE gpurun call, waiting for a free GPU slot: resubmits only while
# gpurun reports that no slot / box is free (status=transient: nothing ran,
# nothing charged). Any other outcome (including a failed GPU step) ends it.
#   bash tools/gpurun_wait.sh <timeout_s> <log> '<command>'
t=$1; log=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log"; then sleep 90; continue; fi
  exit $rc
done
exit 3
