#!/bin/bash
# gpurun, retried only while no GPU slot is free (exit code 3: nothing ran,
# nothing charged); any other outcome ends it.  Usage: tools/gpurun_wait.sh LIMIT 'COMMAND'
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no slot free, retrying in 120 s ($i)"
  sleep 120
done
exit 3
