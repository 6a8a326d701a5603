#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports no free box / slot (nothing ran,
# nothing charged). Any call that actually ran ends the loop, whatever its result.
# usage: tools/gpu_submit.sh LOG TIMEOUT_S 'command'
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && grep -q "run 0.0s\|run Nones" "$log"; then
    echo "[submit] attempt $i: no box ($(grep -o 'all .* busy\|no free box\|backing off' "$log" | head -1)); retry in 120 s" >> "$log.tries"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
