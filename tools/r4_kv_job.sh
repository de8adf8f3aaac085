#!/bin/bash
# GPU box job (round 4): kernel-form A/B on the ICP alone (16 rounds) and on the bench step
# (interleaved bench lines per form).  usage: bash tools/r4_kv_job.sh TAG "forms"
set -u
TAG=$1; VARS=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
ICP_CONFIG=config4 AB_ROUNDS=16 timeout -k 10 300 python -u tools/icp_var_ab.py $VARS > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in $VARS; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-variant $v > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { echo "bench $v failed"; tail -5 $OUT/b_${v}_$r.err; exit 1; }
  python - $OUT/b_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("form", sys.argv[2], "ms/step %.3f icp %.3f gn/iter %.4f" % (d["ms_per_step"], d["icp_kernel_ms"], d["ms_per_gn_iter"]))
PY
done; done
