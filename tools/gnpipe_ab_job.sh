#!/bin/bash
# GPU box job: pipelined (default) vs host-decided GN loop (DPG_GN_PIPE=0), alternated in bench.py,
# after the GN tests.  usage: bash tools/gnpipe_ab_job.sh TAG [test files...]
set -u
OUT=gpurun_out/${1:-gnpipe}; shift; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
T=${*:-tests/test_gpu_solver.py}
timeout -k 10 400 python -u -m pytest $T -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -2 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
MODES=${MODES:-"0 1"}
for r in 1 2 3; do
  for m in $MODES; do   # "P" or "PgG": DPG_GN_PIPE=P, DPG_GATHER_G=G
    G=4; case $m in *g*) G=${m#*g};; esac
    DPG_GN_PIPE=${m%%g*} DPG_GATHER_G=$G timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${m}_$r.json 2> $OUT/b_${m}_$r.err || exit $?
    python - $OUT/b_${m}_$r.json pipe=$m <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms/step %.3f" % d["ms_per_step"], "ms/gn-iter %.4f" % d["ms_per_gn_iter"], "iters", d["gn_iterations"], "fact", d["gn_factorizations"], "err %.12e" % d["final_error"], "icp %.3f" % d["icp_kernel_ms"])
PY
  done
done
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 7 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
  f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats.csv
  python - $OUT/kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:24]:
    print("%-44s %6s calls  avg %9.1f us  total %8.3f ms" % (r["Name"].split("(")[0][-44:], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
fi
