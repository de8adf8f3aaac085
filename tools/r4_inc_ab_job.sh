#!/bin/bash
# incremental line, two builds alternating (DPGSLAM_LIB): usage: bash tools/r4_inc_ab_job.sh ROUNDS LIB_A LIB_B ...
set -u
R=$1; shift
for r in $(seq 1 "$R"); do
  for L in "$@"; do
    DPGSLAM_LIB=$L timeout -k 10 200 python -u bench.py --workload incremental --no-cpu-baseline > gpurun_out/incab.json 2>/dev/null || exit 1
    python -c "import json,sys;d=json.load(open('gpurun_out/incab.json'));t=d['tail_breakdown_ms'];print(sys.argv[1], round(d['p50_ms'],4), round(d['p90_ms'],4), round(d['nodes_per_s_tail'],1), round(t['symbolic_host'],4), t['symbolic_parts'])" "$L"
  done
done
