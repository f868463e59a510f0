#!/bin/bash
# gpurun, re-queued while the pool has no free slot / box (status=transient: nothing ran, nothing
# charged).  Any other outcome -- success or failure of the command -- ends it.
# Usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  if grep -q "status=transient" "$out"; then sleep 150; continue; fi
  break
done
