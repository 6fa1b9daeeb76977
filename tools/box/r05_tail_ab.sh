#!/bin/bash
# Round 5: signed PUT hashing near the end of the body.  TRITONDL_SHA_MB_TAIL
# chunks at the end are hashed in pairs; with frontier-aware claims (default)
# is the 32-chunk tail still needed, and would all-pairs (160 = the whole
# 10 MiB) shorten the 0.4-0.5 ms tail?
set -o pipefail
OUT=${OUT:-gpurun_out/r05_tail_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b tail32_$i && TRITONDL_SHA_MB_TAIL=160 b tail160_$i && TRITONDL_SHA_MB_TAIL=0 b tail0_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1 | grep -o '"get_pump_end": [0-9.]*, "put_sent": [0-9.]*')"
done
exit $rc
