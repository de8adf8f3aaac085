#!/bin/bash
# GPU box job (round 6): angular ICP kernel-form A/B (tools/icp_var_ab.py, byte-identical check) on
# configs 4 and 2, then the candidate counters of each form (lib/libdpg_stats.so).
# usage: bash tools/r6_ab_job.sh TAG variants...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for cfg in config4 config2; do
  ICP_CONFIG=$cfg AB_ROUNDS=${AB_ROUNDS:-6} timeout -k 10 300 python -u tools/icp_var_ab.py "$@" > $OUT/ab_$cfg.txt 2>&1
  rc=$?; cat $OUT/ab_$cfg.txt; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${STATS:-}" ]; then
  for v in "$@"; do
    DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_stats.so timeout -k 10 200 python -u tools/icp_stats.py --variant $v > $OUT/stats_$v.txt 2>&1
    rc=$?; cat $OUT/stats_$v.txt; [ $rc -eq 0 ] || exit $rc
  done
fi
