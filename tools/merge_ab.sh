#!/bin/bash
# GPU box job: the Cholesky alone (tools/build/chol_bench, configs 3 and 4) with the supernode merge
# rule A/B (DPG_CHOL_MERGE_ANY=1: a column joins its child's supernode whatever its other
# children), the timing build's critical paths for both.  usage: bash tools/merge_ab.sh TAG
set -u
TAG=${1:-merge}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for c in 4 3; do
  for M in 0 1; do
    if [ "$M" = 1 ]; then export DPG_CHOL_MERGE_ANY=1; else unset DPG_CHOL_MERGE_ANY; fi
    timeout -k 10 60 tools/build/chol_bench tools/build/pairs$c.bin 40 > "$OUT/c${c}_M$M.log" 2>&1; rc=$?
    echo "config$c merge_any=$M rc=$rc $(cat $OUT/c${c}_M$M.log)"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 60 tools/build/chol_bench_t tools/build/pairs$c.bin 3 > "$OUT/timing${c}_M$M.log" 2>&1; rc=$?
    echo "timing rc=$rc"; grep -E "span|critical" "$OUT/timing${c}_M$M.log"; [ $rc -eq 0 ] || exit $rc
  done
done
