#!/bin/bash
# GPU box job: the prepare's symbolic half on a worker thread (DPG_INC_ASYNC=1 default / 0) on the
# incremental line (config 4, V = 5000) and the config-5 DpgSLAM run, then the full GPU suite.
# usage: bash tools/incasync_ab_job.sh TAG
set -u
TAG=${1:-incasync}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for a in 1 0 1; do
  DPG_INC_ASYNC=$a timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > $OUT/inc_a$a.json 2> $OUT/inc_a$a.err
  rc=$?; echo "inc async=$a exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('$OUT/inc_a$a.json')); print('inc async=$a', {k: round(d[k],3) for k in ('p50_ms','p90_ms','mean_ms_all','nodes_per_s_tail')}, {k: (round(v,3) if not isinstance(v,dict) else v) for k,v in d['tail_breakdown_ms'].items()})"
done
for a in 1 0; do
  DPG_INC_ASYNC=$a timeout -k 10 300 python -u bench.py --workload dynamic --no-cpu-baseline > $OUT/c5_a$a.json 2> $OUT/c5_a$a.err
  rc=$?; echo "c5 async=$a exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$OUT/c5_a$a.json')); print('c5 async=$a', round(d['value'],1), 'nodes/s', {k: round(v,3) for k, v in d['node_ms'].items() if not isinstance(v, dict)}, [round(x['ms'],1) for x in d['sweeps']])"
done
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -2 $OUT/tests.log; exit $rc
