#!/bin/bash
# GPU box job: the incremental reorder rule A/B (DPG_INC_ND: 0 round 2's rule, 2 the 2-start
# search, -1 the batch analysis's pick by critical-path estimate) on the incremental line (config 4,
# V = 5000) and the config-5 DpgSLAM run, then tests/test_inc.py under the new rule.
# usage: bash tools/incnd_ab_job.sh TAG
set -u
TAG=${1:-incnd}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for v in "0 64" "2 64" "-1 64" "-1 32"; do set -- $v; nd=$1; re=$2
  DPG_INC_ND=$nd timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 --inc-reorder-every $re > $OUT/inc_nd${nd}_re$re.json 2> $OUT/inc_nd${nd}_re$re.err
  rc=$?; echo "inc nd=$nd re=$re exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('$OUT/inc_nd${nd}_re$re.json')); print('inc nd=$nd re=$re', {k: round(d[k],3) for k in ('p50_ms','p90_ms','mean_ms_all','nodes_per_s_tail')}, {k: (round(v,3) if not isinstance(v,dict) else v) for k,v in d['tail_breakdown_ms'].items()})"
done
for nd in 0 2 -1; do
  DPG_INC_ND=$nd timeout -k 10 300 python -u bench.py --workload dynamic --no-cpu-baseline > $OUT/c5_nd${nd}.json 2> $OUT/c5_nd${nd}.err
  rc=$?; echo "c5 nd=$nd exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$OUT/c5_nd${nd}.json')); print('c5 nd=$nd', round(d['value'],1), 'nodes/s', {k: round(v,3) for k, v in d['node_ms'].items() if not isinstance(v, dict)}, [round(x['ms'],1) for x in d['sweeps']])"
done
DPG_INC_ND=-1 timeout -k 10 600 python -u -m pytest tests/test_inc.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -2 $OUT/tests.log; exit $rc
