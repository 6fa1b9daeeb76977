#!/bin/bash
# Heap policy A/B on the big-buffer paths: a 2 GiB magnet download from 4
# local seeders and the 1 GiB http job, glibc's dynamic mmap threshold vs the
# fixed 256 KiB default, alternated.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_malloc_big}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for t in 0 262144; do
    timeout -k 10 200 python tools/bench_bt.py --mb 2048 --seeds 4 --malloc-mmap-threshold $t >> $OUT/bt_$t.log 2>&1 || exit $?
  done
done
for rep in 1 2; do
  for t in 0 262144; do
    TRITONDL_MALLOC_MMAP_THRESHOLD=$t timeout -k 10 300 python bench.py --file-mb 1024 --steps 5 --warmup 1 --no-gpu-probe >> $OUT/big_$t.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
