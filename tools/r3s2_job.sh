#!/bin/bash
# GPU box job (round 3, session 2): selected GPU tests, then the ICP cost-predictability probe.
# usage: bash tools/r3s2_job.sh TAG [test files...]
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  echo "tests exit $rc"; tail -3 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head -20; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u tools/icp_cost_predict.py config4 > $OUT/cost_predict.txt 2>&1; rc=$?; cat $OUT/cost_predict.txt; exit $rc
