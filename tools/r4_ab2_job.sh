#!/bin/bash
# GPU box job (round 4): ICP kernel variant A/B on config 4 and config 2 (byte-identical asserted),
# then the cooperative-queue threshold sweep on config 4.  usage: bash tools/r4_ab2_job.sh TAG "variants" "caps"
set -u
TAG=$1; VARS=$2; CAPS=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for cfg in config4 config2; do
  ICP_CONFIG=$cfg AB_ROUNDS=${AB_ROUNDS:-8} timeout -k 10 300 python -u tools/icp_var_ab.py $VARS > $OUT/ab_$cfg.txt 2>&1; rc=$?
  echo "== $cfg"; cat $OUT/ab_$cfg.txt; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$CAPS" ]; then
  ICP_CONFIG=config4 AB_ROUNDS=${AB_ROUNDS:-8} timeout -k 10 300 python -u tools/icp_cap_ab.py $CAPS > $OUT/cap.txt 2>&1; rc=$?
  echo "== caps"; cat $OUT/cap.txt; exit $rc
fi
