#!/bin/bash
# L11^-1 A/B on the config-4 pattern: the Cholesky alone at several solve_inv_cols (0 = off) + kernel times
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; OUT=$ROOT/gpurun_out/${1:-inv}; mkdir -p "$OUT"; cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
python tools/make_pairs.py config4 "$OUT/pairs.bin" || exit 1
for v in 0 48 96 150 0 48; do
  timeout -k 10 60 tools/build/chol_bench "$OUT/pairs.bin" 20 $v > "$OUT/chol_$v.log" 2>&1 || exit 1
  echo "inv_cols=$v $(tail -1 $OUT/chol_$v.log)"
done
for v in 48 150; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o run --output-format csv -- \
      tools/build/chol_bench "$OUT/pairs.bin" 5 $v > /dev/null 2>&1 || exit 1
  echo "== $v"; python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof_$v/run_kernel_stats.csv')):
    print(r['Name'].replace('(anonymous namespace)::','')[:28], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
done
