#!/bin/bash
# GPU box job: config-5 DpgSLAM run (bench.py --workload dynamic) with the incremental reorder rule
# A/B (DPG_INC_ND=0: round 2's separator rule; 2: the 2-start search), interleaved twice.
# usage: bash tools/c5_ab_job.sh TAG
set -u
TAG=${1:-c5ab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for r in 1 2; do for nd in 0 2; do
  DPG_INC_ND=$nd timeout -k 10 300 python -u bench.py --workload dynamic --no-cpu-baseline > $OUT/c5_nd${nd}_r$r.json 2> $OUT/c5_nd${nd}_r$r.err
  rc=$?; echo "c5 nd=$nd round $r exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$OUT/c5_nd${nd}_r$r.json')); print('nd=$nd', round(d['value'],1), 'nodes/s', {k: round(v,3) for k, v in d['node_ms'].items() if not isinstance(v, dict)}, [round(x['ms'],1) for x in d['sweeps']])"
done; done
