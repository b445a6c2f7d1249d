#!/bin/bash
# Submit one gpurun call; while the pool has no box for it (nothing ran, nothing charged:
# "no free box", "busy", "transient" infrastructure verdicts) wait and submit the same call
# again.  A call that ran -- passed or failed -- is never resubmitted.
# usage: tools/gpurun_wait.sh OUT_FILE SCRIPT [TIMEOUT_S]
out=$1; script=$2; to=${3:-1200}
for i in $(seq 1 12); do
  timeout $((to + 1800)) /usr/local/graft/bin/gpurun --timeout "$to" -- bash "$script" > "$out" 2>&1
  if grep -q -E "no free box|slot\(s\) on this pod are busy|status=transient" "$out"; then
    echo "[wait] attempt $i: no box, retrying" >> "$out.attempts"
    if grep -q "backing off" "$out"; then sleep 480; else sleep 150; fi
    continue
  fi
  break
done
