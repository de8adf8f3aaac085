#!/bin/bash
# GPU box job (round 4): incremental-path GPU tests, the incremental bench line and the config-5 line.
# usage: bash tools/r4_inc_job.sh TAG [test files...]
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  echo "tests exit $rc"; grep -E "passed|failed" $OUT/tests.log | tail -3
  [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $OUT/tests.log | tail -80; exit $rc; }
fi
timeout -k 10 300 python -u bench.py --workload incremental > $OUT/inc.json 2> $OUT/inc.err || { echo "inc failed"; tail -20 $OUT/inc.err; exit 1; }
python - $OUT/inc.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("inc p50 %.3f p90 %.3f nodes/s %.1f" % (d["p50_ms"], d["p90_ms"], d["nodes_per_s_tail"]), json.dumps(d.get("tail_breakdown_ms")))
PY
if [ "${C5:-0}" = 1 ]; then
  timeout -k 10 400 python -u bench.py --workload dynamic > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail -20 $OUT/c5.err; exit 1; }
  python - $OUT/c5.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c5 nodes/s %.1f" % d["value"], {k: d[k] for k in d if "p50" in k or "p90" in k})
PY
fi
