#!/bin/bash
# GPU box job: the ISAM2 update's assembly before the Cholesky upload (DPG_INC_EARLY_ASM=1 / 0)
# on the incremental line and the config-5 run, interleaved; then tests/test_inc.py + test_slam.py
# usage: bash tools/incearly_ab_job.sh TAG
set -u
TAG=${1:-incearly}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for r in 1 2; do for e in 1 0; do
  DPG_INC_EARLY_ASM=$e timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > $OUT/inc_e${e}_$r.json 2> $OUT/inc_e${e}_$r.err
  rc=$?; [ $rc -eq 0 ] || { echo "inc exit $rc"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$OUT/inc_e${e}_$r.json')); print('inc early=$e', {k: round(d[k],3) for k in ('p50_ms','p90_ms','mean_ms_all','nodes_per_s_tail')}, 'numeric', round(d['tail_breakdown_ms']['numeric'],3))"
done; done
for e in 1 0; do
  DPG_INC_EARLY_ASM=$e timeout -k 10 300 python -u bench.py --workload dynamic --no-cpu-baseline > $OUT/c5_e$e.json 2> $OUT/c5_e$e.err
  rc=$?; [ $rc -eq 0 ] || { echo "c5 exit $rc"; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/c5_e$e.json')); print('c5 early=$e', round(d['value'],1), 'nodes/s', {k: round(v,3) for k, v in d['node_ms'].items() if not isinstance(v, dict)})"
done
DPG_INC_EARLY_ASM=1 timeout -k 10 600 python -u -m pytest tests/test_inc.py tests/test_slam.py tests/test_adapter.py tests/test_config5.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -1 $OUT/tests.log; exit $rc
