#!/bin/bash
# GPU box job: tools/build/chol_bench on configs 4 and 3 for supernode shapes "MAXCOLS:RELAX" in
# SNLIST (DPG_CHOL_MAXCOLS / DPG_CHOL_RELAX).  usage: SNLIST="64:0.3 32:0.3" bash tools/sn_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$PWD}"
for sn in ${SNLIST:-64:0.3}; do
  export DPG_CHOL_MAXCOLS=${sn%%:*} DPG_CHOL_RELAX=${sn##*:}
  for c in 4 3; do
    out=$(timeout -k 10 60 tools/build/chol_bench tools/build/pairs$c.bin 40); rc=$?
    echo "sn=$sn config$c rc=$rc $out"; [ $rc -eq 0 ] || exit $rc
  done
done
