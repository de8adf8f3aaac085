#!/bin/bash
# config-5 DpgSLAM line with two builds of libdpg.so on one box, alternating (A B A B)
# usage: bash tools/c5_lib_ab.sh TAG libA.so libB.so
set -u
TAG=$1; A=$2; B=$3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do
  for L in "$A" "$B"; do
    n=$(basename "$L" .so)
    DPGSLAM_LIB=$L timeout -k 10 300 python -u bench.py --workload dynamic > "$OUT/c5_${n}_$r.json" 2> "$OUT/c5_${n}_$r.err" || exit $?
    python3 -c "
import json,sys; d=json.loads(open('$OUT/c5_${n}_$r.json').read().strip().splitlines()[-1])
print('$n run $r', round(d['value'],1), 'nodes/s; p50', round(d['node_ms']['p50'],3), 'p90', round(d['node_ms']['p90'],3), 'sweeps', [round(s['ms'],1) for s in d['sweeps']])"
  done
done
