#!/bin/bash
# GPU box job (round 6): kernel trace of the N = 8 shard probe (tools/icp_lpt_probe.py), to see the
# split launch's head and rest kernels.  usage: bash tools/r6_lpt_trace_job.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${1:-r6lpt}
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
PROBE_N=8 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- \
    python3 tools/icp_lpt_probe.py config4 3 > $OUT/probe.txt 2>&1
rc=$?; cat $OUT/probe.txt; exit $rc
