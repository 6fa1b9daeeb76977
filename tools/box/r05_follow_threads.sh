#!/bin/bash
# Round 5: with frontier-aware claims (pairs at the receive frontier), do more
# chunk hashers shorten the signed PUT's tail?  4 (default) vs 6 vs 8.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_follow_threads}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b s4_$i --sign-threads 4 && b s6_$i --sign-threads 6 && b s8_$i --sign-threads 8 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1 | grep -o '"get_pump_end": [0-9.]*, "put_sent": [0-9.]*')"
done
exit $rc
