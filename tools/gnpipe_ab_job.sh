#!/bin/bash
# GPU box job: pipelined (default) vs host-decided GN loop (DPG_GN_PIPE=0), alternated in bench.py,
# after the GN tests.  usage: bash tools/gnpipe_ab_job.sh TAG [test files...]
set -u
OUT=gpurun_out/${1:-gnpipe}; shift; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
T=${*:-tests/test_gpu_solver.py}
timeout -k 10 400 python -u -m pytest $T -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests exit $rc"; tail -2 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for m in 0 1; do
    DPG_GN_PIPE=$m timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${m}_$r.json 2> $OUT/b_${m}_$r.err || exit $?
    python - $OUT/b_${m}_$r.json pipe=$m <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms/step %.3f" % d["ms_per_step"], "ms/gn-iter %.4f" % d["ms_per_gn_iter"], "iters", d["gn_iterations"], "fact", d["gn_factorizations"], "err %.12e" % d["final_error"], "icp %.3f" % d["icp_kernel_ms"])
PY
  done
done
