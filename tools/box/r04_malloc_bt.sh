#!/bin/bash
# Heap policy on the magnet path, more alternations: 2 GiB from 4 local
# seeders, glibc's dynamic mmap threshold vs the fixed 256 KiB default.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_malloc_bt}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3 4 5 6; do
  for t in 0 262144; do
    timeout -k 10 200 python tools/bench_bt.py --mb 2048 --seeds 4 --malloc-mmap-threshold $t >> $OUT/bt_$t.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
