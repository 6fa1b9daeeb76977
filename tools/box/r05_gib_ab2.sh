#!/bin/bash
# Round 5: batching only when one signed PUT pump is running.  1 GiB job
# (4 parts in flight: no batching now) vs batching off entirely, and the
# 10 MiB headline (one PUT: batched) vs batching off.  Alternated runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_gib_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 240 python bench.py --no-gpu-probe --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b gib_now_$i --file-mb 1024 --steps 6 --warmup 1 &&
  TRITONDL_ZC_WRITE_BATCH=0 b gib_nobatch_$i --file-mb 1024 --steps 6 --warmup 1 &&
  b small_now_$i --steps 300 --warmup 10 &&
  TRITONDL_ZC_WRITE_BATCH=0 b small_nobatch_$i --steps 300 --warmup 10 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f | head -1)"
done
exit $rc
