#!/bin/bash
# Placement check on a fresh lease: the NUMA node of every L3 domain, the
# driver's bench command FIRST, then 300-job runs alternating cleanup on/off,
# each reporting where its rank and fakes landed (diag.fake_ccd,
# diag.fakes_same_numa_node).
set -o pipefail
OUT=${OUT:-gpurun_out/r04_fresh5}
mkdir -p $OUT
export TMPDIR=/tmp
python3 -c "
from tritondl.parallel import topology as t
print({d[0]: t.numa_node_of(d[0]) for d in t.l3_domains()})" > $OUT/numa.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 &&
for arm in on off on off on off; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cleanup $arm >> $OUT/ab_$arm.log 2>&1 || exit $?
done &&
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-gpu-probe >> $OUT/driver_again.log 2>&1 || exit $?
done
rc=$?
cat $OUT/numa.txt
for f in $OUT/bench_driver.log $OUT/ab_*.log $OUT/driver_again.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"
done
exit $rc
