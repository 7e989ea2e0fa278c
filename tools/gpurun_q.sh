#!/bin/bash
# Queue wrapper (development): runs one gpurun call, retrying ONLY while gpurun reports that no
# box or slot was free (exit 3, nothing ran, nothing charged).  Usage: tools/gpurun_q.sh LOG TIMEOUT CMD
LOG=$1; TO=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "GPU slot(s) on this pod are busy" "$LOG"; then break; fi
  sleep 150
done
echo "rc=$rc" >> "$LOG"
exit $rc
