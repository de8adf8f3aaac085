#!/bin/bash
# GPU box job: in-process A/B of angular ICP kernel variants (byte-identical results asserted).
# usage: bash tools/r4_ab_job.sh TAG "variants" [config]
set -u
TAG=$1; VARS=$2; CFG=${3:-config4}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
ICP_CONFIG=$CFG AB_ROUNDS=${AB_ROUNDS:-6} timeout -k 10 400 python -u tools/icp_var_ab.py $VARS > $OUT/ab_$CFG.txt 2>&1; rc=$?; cat $OUT/ab_$CFG.txt; exit $rc
