#!/bin/bash
# usage: gpurun_retry.sh LOG TIMEOUT 'command'  -- retries ONLY when no GPU slot/box was free (nothing ran)
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "no free box right now\|GPU slot(s) on this pod are busy" $LOG && [ $rc -ne 0 ]; then
    sleep 150; continue
  fi
  exit $rc
done
