#!/bin/bash
# One GPU-box session of several steps (run from the repo root via gpurun):
#   bash tools/gpu_session.sh TAG "step1 cmd" "step2 cmd" ...
# Each step runs under its own `timeout -k 10 <STEP_TIMEOUT>` with output to
# gpurun_out/<TAG>_<i>.log.  An ordinary failure (exit 1: a failed test) lets the session go
# on; a timeout, abort, fault or signal (any other non-zero status) ends it there, so nothing
# more touches the GPU after trouble.
TAG=$1
shift
STEP_TIMEOUT=${STEP_TIMEOUT:-600}
mkdir -p gpurun_out
i=0
worst=0
for cmd in "$@"; do
  i=$((i + 1))
  log=gpurun_out/${TAG}_${i}.log
  echo "== step $i: $cmd" | tee "$log"
  timeout -k 10 "$STEP_TIMEOUT" bash -c "$cmd" >> "$log" 2>&1
  rc=$?
  echo "== step $i rc=$rc" | tee -a "$log"
  tail -3 "$log"
  if [ $rc -gt 1 ]; then
    echo "stopping after step $i (rc=$rc)"
    exit $rc
  fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
