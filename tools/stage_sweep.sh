#!/bin/bash
# GPU box job: tools/build/chol_bench on configs 4 and 3 for each solve staging size in RLIST
# (DPG_SOLVE_STAGE, doubles; "default" = the library's choice).  usage: RLIST="0 default" bash tools/stage_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$PWD}"
for R in ${RLIST:-0 default}; do
  if [ "$R" = default ]; then unset DPG_SOLVE_STAGE; else export DPG_SOLVE_STAGE=$R; fi
  for c in 4 3; do
    out=$(timeout -k 10 60 tools/build/chol_bench tools/build/pairs$c.bin 40); rc=$?
    echo "R=$R config$c rc=$rc $out"; [ $rc -eq 0 ] || exit $rc
  done
done
