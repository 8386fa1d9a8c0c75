# Submit ONE gpurun call, waiting for a free GPU slot: re-submits only while gpurun answers
# "no box / slot free" or "backing off" (exit code 3 or a transient status: nothing ran,
# nothing was charged); any call that ran — pass or fail — ends the loop.  Never retries a
# command that ran on the GPU.
#   bash tools/gpu_call.sh <log> <timeout-s> '<command>'
LOG=$1
TMO=$2
CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|already running" "$LOG" && ! grep -q "status=ok" "$LOG"; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
