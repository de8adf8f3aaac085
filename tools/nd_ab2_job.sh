#!/bin/bash
# GPU box job: separator-cover A/B.  tools/chol_bench on the config-4 / config-3 patterns with the
# batch pick and single candidates, cover refinement on (default) and off (DPG_ND_NOCOVER); then the
# incremental bench with the default reorder rule, cover on and off.  usage: bash tools/nd_ab2_job.sh TAG
set -u
TAG=${1:-nd2}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
for c in config4 config3; do python tools/make_pairs.py $c "$OUT/$c.bin" || exit 1; done
for round in 1 2; do
  for c in config4 config3; do
    for k in pick 0 2 3; do
      for cov in on off; do
        [ "$k" = "0" ] && [ "$cov" = "off" ] && continue
        echo -n "round $round $c nd=$k cover=$cov: "
        env $( [ "$k" != pick ] && echo DPG_CHOL_ND=$k ) $( [ "$cov" = off ] && echo DPG_ND_NOCOVER=1 ) \
          timeout -k 10 120 tools/build/chol_bench "$OUT/$c.bin" 20 2>&1 | tail -1
        rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
      done
    done
  done
done | tee "$OUT/nd_ab2.txt"
for cov in on off; do
  env $( [ "$cov" = off ] && echo DPG_ND_NOCOVER=1 ) timeout -k 10 300 python -u bench.py --workload incremental > $OUT/inc_cover_$cov.json 2> $OUT/inc_cover_$cov.err
  rc=$?; echo "inc cover=$cov exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$OUT/inc_cover_$cov.json')); print('cover=$cov', {k: round(d[k],3) for k in ('p50_ms','p90_ms','mean_ms_all')}, 'numeric', round(d['tail_breakdown_ms']['numeric'],3))"
done
