#!/bin/bash
# usage: tools/gpurun_queue.sh <out-file> <gpurun args...>   (run from the repo root; the GPU command itself never retries)
# gpurun, re-queued ONLY while the pool has no free slot (exit 3: nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "slot(s) on this pod are busy" "$out"; then break; fi
  sleep 90
done
echo "rc=$rc" >> "$out"
echo done >> "$out"
