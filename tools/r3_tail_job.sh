#!/bin/bash
# GPU box job: GPU suite + incremental line + config-5 run + the 2-rank (gloo, one card) bench rehearsal
# usage: bash tools/r3_tail_job.sh TAG
set -u
TAG=${1:-tail}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > $OUT/inc_$r.json 2> $OUT/inc_$r.err
  rc=$?; echo "inc exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('$OUT/inc_$r.json')); print('inc', {k: round(d[k],3) for k in ('p50_ms','p90_ms','mean_ms_all','nodes_per_s_tail')}, d['tail_breakdown_ms'])"
done
timeout -k 10 300 python -u bench.py --workload dynamic --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err
rc=$?; echo "c5 exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/c5.json')); print('c5', round(d['value'],1), 'nodes/s', {k: round(v,3) for k, v in d['node_ms'].items() if not isinstance(v, dict)})"
bash tools/dist_job.sh $TAG/dist
