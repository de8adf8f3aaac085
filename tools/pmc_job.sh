#!/bin/bash
# GPU box job: PMC counters for one bench step (each counter group in its own rocprofv3 pass,
# kernel trace only beside --pmc).  usage: bash tools/pmc_job.sh TAG
set -u
TAG=${1:-pmc}
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONPATH=$ROOT:$ROOT/dpg-slam_amd
export TMPDIR=/tmp
run() {   # name, counters...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
        python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name exit $rc"
    return $rc
}
# provenance: the hash of the ICP kernel's sources as they ran here (bench.py kernel_src_sha256)
python3 -c "import bench; print(bench.kernel_src_sha256())" > "$OUT/src.sha256"
[ -f BUILD_GIT_SHA ] && cp BUILD_GIT_SHA "$OUT/git.sha"
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE && \
run lds SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
