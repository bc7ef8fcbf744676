#!/bin/bash
# usage: tools/gpuq.sh LOG TIMEOUT CMD  -- retries only when gpurun reports no free slot (exit 3)
LOG=$1; TO=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "busy .* nothing was charged" $LOG; then break; fi
  sleep 150
done
echo "done rc=$rc" >> $LOG
