#!/bin/bash
# GPU box job: the bench step's stream priority A/B (DPG_BENCH_STREAM_PRIO=high / normal), interleaved
# usage: bash tools/prio_ab_job.sh TAG
set -u
TAG=${1:-prio}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
for r in 1 2; do for pr in high normal; do
  DPG_BENCH_STREAM_PRIO=$pr timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_${pr}_$r.json 2> $OUT/b_${pr}_$r.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $pr exit $rc"; tail -5 $OUT/b_${pr}_$r.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/b_${pr}_$r.json')); print('$pr', 'ms/step %.3f gn %.4f icp %.3f cov %.3f err %.12e' % (d['ms_per_step'], d['ms_per_gn_iter'], d['icp_kernel_ms'], d['cov_kernel_ms'], d['final_error']))"
done; done
