#!/bin/bash
# GPU box job (round 6): the rank form at world 2 on one card over gloo (tools/rank_check.py,
# config 4), the blocking host collective (previous build) against the collective thread, 2 rounds.
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${1:-r6hc}
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd:$ROOT/tests
for r in 1 2; do
  for L in dpg-slam_amd/lib/libdpg_blockinghc.so dpg-slam_amd/lib/libdpg.so; do
    DPGSLAM_LIB=$L timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $((29600 + r)) tools/rank_check.py config4 > $OUT/rc.log 2>&1
    rc=$?; echo "$L: $(grep -h 'rank check ok' $OUT/rc.log | sed 's/.*gn ms/gn ms/' | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -20 $OUT/rc.log; exit $rc; }
  done
done
