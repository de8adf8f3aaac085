#!/bin/bash
# GPU box job: the batch symbolic analysis' separator rules (dpg_chol_symbolic candidates,
# DPG_CHOL_ND=k) timed by tools/chol_bench on the config-4 and config-3 patterns, two interleaved
# rounds.  usage: bash tools/nd_ab_job.sh TAG
set -u
TAG=${1:-nd}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
for c in config4 config3; do python tools/make_pairs.py $c "$OUT/$c.bin" || exit 1; done
for round in 1 2; do
  for c in config4 config3; do
    for k in 0 1 2 3; do
      echo -n "round $round $c nd=$k: "
      DPG_CHOL_ND=$k timeout -k 10 120 tools/build/chol_bench "$OUT/$c.bin" 20 2>&1 | tail -1
      rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
    done
  done
done | tee "$OUT/nd_ab.txt"
