#!/bin/bash
# GN refactor policy sweep: dpg_gn_params.refactor_delta (chord steps once max|delta| falls below
# it, while they contract >= 10x) on the config-4 bench step and on the config-5 run's sweeps
# (bench.py --workload dynamic, 2 passes); stops at the first failure.
mkdir -p gpurun_out
out=gpurun_out/refactor_sweep.txt
: > $out
for d in ${1:-1e-4 1e-3 1e-2}; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --refactor-delta $d > gpurun_out/rs.json 2>/dev/null || { echo "delta $d failed" >> $out; exit 1; }
  python -c "
import json; b=json.load(open('gpurun_out/rs.json'))
print('refactor_delta $d', 'ms/step %.3f' % b['ms_per_step'], 'gn_iter %s' % b['gn_iterations'], 'fact %s' % b['gn_factorizations'], 'ms/gn_iter %.3f' % b['ms_per_gn_iter'])" >> $out
done
