#!/bin/bash
# Client-side retry of a gpurun call while the pool has no box (transient / backing off):
# nothing ran on a GPU in those attempts.  usage: tools/gpurun_retry.sh <log> <timeout> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  if grep -q "status=transient" $log; then
    w=$(grep -o "retry in [0-9]*s" $log | grep -o "[0-9]*" | tail -1); w=${w:-120}
    [ "$w" -lt 60 ] && w=60
    echo "attempt $i: transient, waiting ${w}s" >> $log.attempts
    sleep $w
    continue
  fi
  break
done
