set -u
OUT=gpurun_out/r3p0; mkdir -p $OUT
export PYTHONPATH=$PWD:$PWD/dpg-slam_amd TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list exit $?"
AB_ROUNDS=3 timeout -k 10 200 python -u tools/icp_ab.py 256 > $OUT/ab.txt 2>&1; echo "ab exit $?"; cat $OUT/ab.txt
