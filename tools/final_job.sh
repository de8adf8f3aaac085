#!/bin/bash
# GPU box job for a round's record: full GPU suite -> smoke -> bench line (with the CPU baselines)
# -> config-2 / config-3 lines -> incremental line -> config-5 DpgSLAM line -> rocprofv3 kernel stats -> PMC passes.
# usage: bash tools/final_job.sh TAG   (every GPU step under its own limit; stops at the first failure)
set -u
TAG=${1:-final}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
cd "$ROOT"
export TMPDIR=/tmp
(nproc; lscpu | head -20) > "$OUT/host.txt" 2>&1
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests exit $rc"; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc"; cat "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
for cfg in config2 config3; do   # "batched ICP + single GN solve" configs: their step and one-off cost
  timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"
  rc=$?; echo "bench $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --workload incremental > "$OUT/inc.json" 2> "$OUT/inc.err"
rc=$?; echo "inc exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload dynamic > "$OUT/c5_dynamic.json" 2> "$OUT/c5_dynamic.err"
rc=$?; echo "dynamic exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_job.sh "$TAG/pmc"
