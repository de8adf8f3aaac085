#!/bin/bash
# GPU box job: ICP kernel variant A/B (config 4 + config 2, byte-identical asserted) and the
# candidate counters of each variant (stats build).  usage: bash tools/r4_var_job.sh TAG "variants"
set -u
TAG=$1; VARS=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for cfg in config4 config2; do
  ICP_CONFIG=$cfg AB_ROUNDS=${AB_ROUNDS:-6} timeout -k 10 400 python -u tools/icp_var_ab.py $VARS > $OUT/ab_$cfg.txt 2>&1; rc=$?; cat $OUT/ab_$cfg.txt; [ $rc -eq 0 ] || exit $rc
done
for v in $VARS; do
  DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_stats.so timeout -k 10 300 python -u tools/icp_stats.py --variant $v > $OUT/stats_v$v.txt 2>&1; rc=$?; echo "== variant $v"; cat $OUT/stats_v$v.txt; [ $rc -eq 0 ] || exit $rc
done
