#!/bin/bash
# GPU box job: Cholesky A/B (inverted diagonal blocks vs substitution chains, tools/build/chol_bench on
# the config-2..4 patterns, both in fresh processes), then the bench line.  usage: bash tools/r3_gn_job.sh TAG
set -u
TAG=${1:-gn}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for c in 3 4; do
  for mode in dinv chain; do
    if [ $mode = chain ]; then export DPG_SOLVE_CHAIN=1; else unset DPG_SOLVE_CHAIN; fi
    timeout -k 10 60 tools/build/chol_bench tools/build/pairs$c.bin 20 > "$OUT/$mode$c.log" 2>&1; rc=$?
    echo "$mode config$c rc=$rc $(cat $OUT/$mode$c.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
unset DPG_SOLVE_CHAIN
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench.json'));print({k:d[k] for k in ('ms_per_step','ms_per_gn_iter','gn_iterations','gn_factorizations','icp_kernel_ms')})"; [ $rc -eq 0 ] || exit $rc
