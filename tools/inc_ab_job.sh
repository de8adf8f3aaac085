#!/bin/bash
# GPU box job: the incremental path's reorder rule A/B (DPG_INC_ND=0: round 2's separator rule,
# default: the 2-start search) on bench.py --workload incremental, then tests/test_inc.py.
# usage: bash tools/inc_ab_job.sh TAG
set -u
TAG=${1:-incab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for nd in 0 2; do
  DPG_INC_ND=$nd timeout -k 10 300 python -u bench.py --workload incremental > $OUT/inc_nd$nd.json 2> $OUT/inc_nd$nd.err
  rc=$?; echo "inc nd=$nd exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('$OUT/inc_nd$nd.json')); print('nd=$nd', {k: d[k] for k in ('p50_ms','p90_ms','mean_ms_all','nodes_per_s_tail')}, d['tail_breakdown_ms'])"
done
timeout -k 10 600 python -u -m pytest tests/test_inc.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -2 $OUT/tests.log; exit $rc
