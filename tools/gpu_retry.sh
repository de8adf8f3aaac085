#!/bin/bash
# retry a gpurun call while the pool has no box (a "transient" verdict: nothing ran, nothing charged);
# stops at any other outcome.  usage: bash tools/gpu_retry.sh LOG TIMEOUT_S 'command'
LOG=$1; shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
for i in $(seq 1 30); do
  rm -f "$ROOT/gpurun_out/.last_call.json"
  bash "$ROOT/tools/gpu.sh" "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q '"status": "transient"' "$ROOT/gpurun_out/.last_call.json" 2>/dev/null || \
     { grep -q "no free box\|slot(s) on this pod are busy\|backing off" "$LOG" && ! grep -q "merged" "$LOG"; }; then
    sleep 120; continue
  fi
  exit $rc
done
