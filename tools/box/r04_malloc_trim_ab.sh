#!/bin/bash
# Pinning glibc's mmap threshold also pins its trim threshold at 128 KiB:
# does per-free() trimming cost the magnet path?  2 GiB from 4 local seeders:
# dynamic (glibc default) vs mmap 256 KiB + trim 128 KiB vs mmap 256 KiB +
# trim 4 MiB vs mmap 1 MiB, alternated; then the headline, trim 128 KiB vs 4 MiB.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_malloc_trim}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  timeout -k 10 200 python tools/bench_bt.py --mb 2048 --seeds 4 --malloc-mmap-threshold 0 >> $OUT/bt_dyn.log 2>&1 || exit $?
  timeout -k 10 200 python tools/bench_bt.py --mb 2048 --seeds 4 --malloc-mmap-threshold 262144 --malloc-trim-threshold 131072 >> $OUT/bt_256k.log 2>&1 || exit $?
  timeout -k 10 200 python tools/bench_bt.py --mb 2048 --seeds 4 --malloc-mmap-threshold 262144 --malloc-trim-threshold 4194304 >> $OUT/bt_256k_trim4m.log 2>&1 || exit $?
  timeout -k 10 200 python tools/bench_bt.py --mb 2048 --seeds 4 --malloc-mmap-threshold 1048576 --malloc-trim-threshold 131072 >> $OUT/bt_1m.log 2>&1 || exit $?
done
for rep in 1 2 3; do
  TRITONDL_MALLOC_TRIM_THRESHOLD=131072 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe >> $OUT/head_256k.log 2>&1 || exit $?
  TRITONDL_MALLOC_TRIM_THRESHOLD=4194304 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe >> $OUT/head_256k_trim4m.log 2>&1 || exit $?
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
