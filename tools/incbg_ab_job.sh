#!/bin/bash
# GPU box job: background reorders A/B (DPG_INC_BG_ORDER=1 default / 0) x the reorder rule
# (DPG_INC_ND 0 / -1) on the incremental line (config 4, V = 5000) and the config-5 DpgSLAM run,
# then tests/test_inc.py (+ the checkpoint and slam tests) under the chosen defaults.
# usage: bash tools/incbg_ab_job.sh TAG
set -u
TAG=${1:-incbg}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for v in "0 1" "-1 1" "-1 0"; do set -- $v; nd=$1; bg=$2
  DPG_INC_ND=$nd DPG_INC_BG_ORDER=$bg timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > $OUT/inc_nd${nd}_bg$bg.json 2> $OUT/inc_nd${nd}_bg$bg.err
  rc=$?; echo "inc nd=$nd bg=$bg exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('$OUT/inc_nd${nd}_bg$bg.json')); print('inc nd=$nd bg=$bg', {k: round(d[k],3) for k in ('p50_ms','p90_ms','mean_ms_all','nodes_per_s_tail')}, {k: (round(v,3) if not isinstance(v,dict) else v) for k,v in d['tail_breakdown_ms'].items()})"
done
for v in "0 1" "-1 1"; do set -- $v; nd=$1; bg=$2
  DPG_INC_ND=$nd DPG_INC_BG_ORDER=$bg timeout -k 10 300 python -u bench.py --workload dynamic --no-cpu-baseline > $OUT/c5_nd${nd}_bg$bg.json 2> $OUT/c5_nd${nd}_bg$bg.err
  rc=$?; echo "c5 nd=$nd bg=$bg exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$OUT/c5_nd${nd}_bg$bg.json')); print('c5 nd=$nd bg=$bg', round(d['value'],1), 'nodes/s', {k: round(v,3) for k, v in d['node_ms'].items() if not isinstance(v, dict)}, [round(x['ms'],1) for x in d['sweeps']])"
done
DPG_INC_ND=-1 timeout -k 10 600 python -u -m pytest tests/test_inc.py tests/test_slam.py tests/test_adapter.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -2 $OUT/tests.log; exit $rc
