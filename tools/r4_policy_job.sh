#!/bin/bash
# GPU box job (round 4): the chord threshold (refactor_delta) -- GN trajectories + bench lines.
set -u
TAG=$1; DELTAS=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 300 python -u tools/gn_delta_trace.py $DELTAS > $OUT/trace.txt 2>&1; rc=$?; cat $OUT/trace.txt; [ $rc -eq 0 ] || exit $rc
for d in $DELTAS; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --refactor-delta $d > $OUT/b_$d.json 2> $OUT/b_$d.err || { echo "bench $d failed"; tail -5 $OUT/b_$d.err; exit 1; }
  python - $OUT/b_$d.json $d <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("refactor_delta", sys.argv[2], "ms/step %.3f icp %.3f gn/iter %.4f iters %.1f fact %.1f err %.12e" % (d["ms_per_step"], d["icp_kernel_ms"], d["ms_per_gn_iter"], d["gn_iterations"], d["gn_factorizations"], d["final_error"]))
PY
done
