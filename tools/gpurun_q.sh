#!/bin/bash
# Queue wrapper (development): runs one gpurun call, retrying ONLY while gpurun reports that no
# box or slot was free (exit 3, nothing ran, nothing charged).  Usage: tools/gpurun_q.sh LOG TIMEOUT CMD
LOG=$1; TO=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  # (retry only when nothing ran: no slot, no free box, or the pool backing off after an
  # infrastructure failure)
  if [ $rc -ne 3 ] && ! grep -qE "GPU slot\(s\) on this pod are busy|no free box|backing off" "$LOG"; then break; fi
  sleep 150
done
echo "rc=$rc" >> "$LOG"
exit $rc
