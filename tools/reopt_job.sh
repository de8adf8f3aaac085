#!/bin/bash
# GPU box: time the reoptimize sweep (tools/reopt_bench.py).  usage: bash tools/reopt_job.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 400 python -u tools/reopt_bench.py config2 3 > "$OUT/reopt.json" 2> "$OUT/reopt.err"
rc=$?; echo "reopt exit $rc"; cat "$OUT/reopt.json"; [ $rc -eq 0 ] || tail -20 "$OUT/reopt.err"; exit $rc
