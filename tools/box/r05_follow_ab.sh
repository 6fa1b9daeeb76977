#!/bin/bash
# Round 5: streamed signed PUT hashers, wide (16-chunk) claims by position
# (TRITONDL_SHA_MB_FOLLOW=0, before) vs only over bytes already downloaded
# (default now); plus the unsigned payload, whose sender now follows the
# download in 256 KiB slices instead of 4 MiB steps.  Alternated 300-job runs
# with the data-plane trace.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_follow_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b follow_$i &&
  TRITONDL_SHA_MB_FOLLOW=0 b position_$i &&
  b unsigned_$i --payload unsigned || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1)"
done
exit $rc
