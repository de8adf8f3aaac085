#!/bin/bash
# GPU box job: reorder period x background-order lead A/B (DPG_INC_REORDER_EVERY, DPG_INC_BG_LEAD)
# on the incremental line (config 4, V = 5000) and the config-5 DpgSLAM run.
# usage: [INC_RE_SET='32:8 16:4'] [C5_RE_SET=...] bash tools/increorder_ab_job.sh TAG  (period:lead pairs)
set -u
TAG=${1:-increorder}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for v in ${INC_RE_SET:-64:16 32:16 32:8 64:8}; do re=${v%%:*}; ld=${v##*:}
  DPG_INC_REORDER_EVERY=$re DPG_INC_BG_LEAD=$ld timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > $OUT/inc_re${re}_l$ld.json 2> $OUT/inc_re${re}_l$ld.err
  rc=$?; echo "inc re=$re lead=$ld exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('$OUT/inc_re${re}_l$ld.json')); print('inc re=$re lead=$ld', {k: round(d[k],3) for k in ('p50_ms','p90_ms','mean_ms_all','nodes_per_s_tail')}, 'numeric', round(d['tail_breakdown_ms']['numeric'],3), 'reorders', d['reorders'])"
done
for v in ${C5_RE_SET:-64:16 32:16 32:8}; do re=${v%%:*}; ld=${v##*:}
  DPG_INC_REORDER_EVERY=$re DPG_INC_BG_LEAD=$ld timeout -k 10 300 python -u bench.py --workload dynamic --no-cpu-baseline > $OUT/c5_re${re}_l$ld.json 2> $OUT/c5_re${re}_l$ld.err
  rc=$?; echo "c5 re=$re lead=$ld exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$OUT/c5_re${re}_l$ld.json')); print('c5 re=$re lead=$ld', round(d['value'],1), 'nodes/s', {k: round(v,3) for k, v in d['node_ms'].items() if not isinstance(v, dict)})"
done
