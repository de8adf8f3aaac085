#!/bin/bash
# GPU box job (round 6): PMC counters of the angular ICP kernel forms given (tools/icp_var_ab.py,
# one round each, config 4), one rocprofv3 pass per counter group; summarised per kernel
# instantiation by tools/pmc_ab_summary.py.  usage: bash tools/r6_pmc_ab_job.sh TAG variants...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
pass() {   # name, counters...
    local name=$1; shift
    AB_ROUNDS=1 ICP_CONFIG=config4 timeout -k 10 150 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run \
        --output-format csv -- python3 tools/icp_var_ab.py $VARS > "$OUT/$name.log" 2>&1
    local rc=$?; echo "$name exit $rc"; return $rc
}
VARS="$*"
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU && \
pass b SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
python3 tools/pmc_ab_summary.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
