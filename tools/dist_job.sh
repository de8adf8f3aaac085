#!/bin/bash
# GPU box: rehearse the multi-rank bench path on one GPU -- 2 ranks sharing the card over gloo
# (the driver's 8-GPU run uses nccl = RCCL).  usage: bash tools/dist_job.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$PWD}; cd "$ROOT"; OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --backend gloo \
    > "$OUT/bench2.json" 2> "$OUT/bench2.err"
rc=$?; echo "dist exit $rc"; cat "$OUT/bench2.json"; [ $rc -eq 0 ] || tail -20 "$OUT/bench2.err"; exit $rc
