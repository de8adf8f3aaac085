#!/bin/bash
# GPU box job: variant A/B of the ICP kernel, then selected GPU test files.
# usage: bash tools/r3_quick_job.sh TAG "variants" [test files...]
set -u
TAG=$1; VARS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
AB_ROUNDS=${AB_ROUNDS:-5} timeout -k 10 300 python -u tools/icp_var_ab.py $VARS > $OUT/ab4.txt 2>&1; rc=$?; cat $OUT/ab4.txt; [ $rc -eq 0 ] || exit $rc
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  echo "tests exit $rc"; tail -3 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head -20; exit $rc
fi
