#!/bin/bash
# A/B of two builds of libdpg on the bench step, alternating in separate processes:
# usage: bash tools/lib_ab.sh ROUNDS LIB_A LIB_B [LIB_C ...]   (prints ms/step, ICP, GN per iteration)
set -u
R=$1; shift
for r in $(seq 1 "$R"); do
  for L in "$@"; do
    DPGSLAM_LIB=$L timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/lib_ab.json 2>/dev/null || exit 1
    python -c "import json,sys;d=json.load(open('gpurun_out/lib_ab.json'));print(sys.argv[1], round(d['ms_per_step'],3), round(d['icp_kernel_ms'],3), round(d['ms_per_gn_iter'],4), d['gn_iterations'], d['final_error'])" "$L"
  done
done
