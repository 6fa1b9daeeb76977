#!/bin/bash
# One worker's capacity beyond the reference's serial model: jobs in flight
# per worker (--concurrency, prefetch equal) 1 / 2 / 4, alternated twice,
# 300 timed jobs each.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_conc}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for c in 1 2 4; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --no-reference-mode --concurrency $c >> $OUT/c$c.log 2>&1 || exit $?
  done
done
for f in $OUT/c*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
