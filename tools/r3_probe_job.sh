#!/bin/bash
# GPU box job: ICP variant A/B, the shard probe, selected GPU tests. usage: bash tools/r3_probe_job.sh TAG "variants" "probe modes" [tests...]
set -u
TAG=$1; VARS=$2; MODES=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
if [ -n "$VARS" ]; then
  AB_ROUNDS=${AB_ROUNDS:-5} timeout -k 10 300 python -u tools/icp_var_ab.py $VARS > $OUT/ab4.txt 2>&1; rc=$?; cat $OUT/ab4.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$MODES" ]; then
  timeout -k 10 300 python -u tools/icp_shard_probe.py $MODES > $OUT/shard.txt 2>&1; rc=$?; cat $OUT/shard.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  echo "tests exit $rc"; tail -3 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head -20; exit $rc
fi
