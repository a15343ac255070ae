#!/bin/bash
# Host-side helper (this container): run one gpurun call, waiting for a free GPU slot.  gpurun exits 3
# when no slot or box is free (nothing ran, nothing charged); only that case is retried, after a pause.
#   bash tools/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1; rc=$?
  [ $rc -eq 3 ] || grep -q "status=transient" "$LOG" || exit $rc
  grep -q "status=transient" "$LOG" || [ $rc -eq 3 ] || exit $rc
  sleep 150
done
exit $rc
