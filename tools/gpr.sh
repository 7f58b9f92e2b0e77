#!/bin/bash
# gpurun with a queue retry (run HERE, not on the box): tools/gpr.sh <log> --timeout S -- <cmd>; reruns only when
# the pool had no free slot (status=transient: nothing ran, nothing charged), at most 8 tries 150 s apart
LOG=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG"; then sleep 150; continue; fi
  break
done
