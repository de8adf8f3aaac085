#!/bin/bash
# GPU box job: tools/icp_var_ab.py on configs 4 (and 3), variants given as arguments.
# usage: bash tools/var_ab_job.sh TAG variants...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
AB_ROUNDS=${AB_ROUNDS:-5} timeout -k 10 300 python -u tools/icp_var_ab.py "$@" > $OUT/ab4.txt 2>&1; rc=$?; cat $OUT/ab4.txt; [ $rc -eq 0 ] || exit $rc
