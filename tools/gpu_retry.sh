#!/bin/bash
# retry a gpurun call while the pool has no box (exit 3 / "no free box" / backoff); stops at any other outcome
# usage: bash tools/gpu_retry.sh LOG TIMEOUT_S 'command'
LOG=$1; shift
for i in $(seq 1 30); do
  bash "$(dirname "$0")/gpu.sh" "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "no free box\|slot(s) on this pod are busy\|backing off" "$LOG" && ! grep -q "merged" "$LOG"; then sleep 150; continue; fi
  exit $rc
done
