#!/bin/bash
# GPU box job (round 4): ICP variant A/B (config 4 + 2, byte-identical) and one PMC pass over the
# same A/B (LDS instructions, bank-conflict cycles, LDS-array cycles, VALU per kernel form).
set -u
TAG=$1; VARS=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
bash tools/r4_ab2_job.sh $TAG "$VARS" || exit 1
AB_ROUNDS=1 ICP_CONFIG=config4 timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES -d $OUT/pmc -o run --output-format csv -- python3 tools/icp_var_ab.py $VARS > $OUT/pmc.log 2>&1
echo "pmc exit $?"
