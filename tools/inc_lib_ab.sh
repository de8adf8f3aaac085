#!/bin/bash
# incremental line with two builds of libdpg.so on one box, alternating (A B A B)
# usage: bash tools/inc_lib_ab.sh TAG libA.so libB.so
set -u
TAG=$1; A=$2; B=$3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do
  for L in "$A" "$B"; do
    n=$(basename "$L" .so)
    DPGSLAM_LIB=$L timeout -k 10 300 python -u bench.py --workload incremental --cpu-nodes 0 > "$OUT/inc_${n}_$r.json" 2> "$OUT/inc_${n}_$r.err" || exit $?
    python3 -c "
import json; d=json.loads(open('$OUT/inc_${n}_$r.json').read().strip().splitlines()[-1]); b=d['tail_breakdown_ms']
print('$n run $r p50', round(d['p50_ms'],4), 'p90', round(d['p90_ms'],4), 'nodes/s', round(d['nodes_per_s_tail'],1), 'numeric', round(b['numeric'],4), 'symbolic', round(b['symbolic_host'],4))"
  done
done
