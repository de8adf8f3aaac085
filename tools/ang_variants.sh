#!/bin/bash
# Build ICP-kernel variants as separate libraries (lib/libdpg_<name>.so) for A/B timing:
#   bash tools/ang_variants.sh name "-DDPG_ANG_KU=8 -DDPG_ANG_WPE=6" [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../dpg-slam_amd"
make -s -j8 all
OBJS=$(ls build/*.o | grep -v -e stats_ -e timing_ -e '/v_' -e dpg_icp_ang.o)
while [ $# -ge 2 ]; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-slp-vectorize -Wall $2 -c csrc/dpg_icp_ang.hip -o build/v_$1.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdpg_$1.so $OBJS build/v_$1.o -lpthread -lm
    echo "lib/libdpg_$1.so"
    shift 2
done
