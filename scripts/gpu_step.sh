#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a fault, abort, segfault
# or timeout (exit 134/139/124/137), continue past ordinary failures (exit 1). A long step
# writes a heartbeat line every 30 s to <logfile>.hb, so a quiet render is not taken for a hang.
# usage: scripts/gpu_step.sh <seconds> <logfile> <command...>
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
echo "### $(date +%T) $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "$log" 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
    sleep 5
    n=$((n + 1))
    [ $((n % 6)) -eq 0 ] && echo "$(date +%T) running" >> "$log.hb"
done
wait $pid
rc=$?
echo "### rc=$rc $*" | tee -a gpurun_out/steps.log
tail -5 "$log"
case $rc in
  0|1|2|5) exit 0 ;;   # success / test failures / usage: keep going
  *) echo "FATAL rc=$rc: stopping GPU work in this call"; exit 99 ;;
esac
