#!/bin/bash
# GPU factor + solve time of the Cholesky under minimum-degree and nested-dissection orders
# (tools/build/chol_bench on the pose-graph patterns bench_in/<graph>_chol.bin); stops at the first
# failure.  usage: order_job.sh "graphs" "orders"
mkdir -p gpurun_out
out=gpurun_out/order_ab.txt
: > $out
for g in ${1:-c4 c5}; do
  for o in ${2:-md nd:32 nd:64}; do
    r=$(DPG_CHOL_ORDER=$o timeout -k 10 60 ./tools/build/chol_bench bench_in/${g}_chol.bin 20) || { echo "$g $o failed: $?" >> $out; exit 1; }
    echo "$g $o: $r" >> $out
  done
done
