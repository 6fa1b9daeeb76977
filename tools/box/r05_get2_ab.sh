#!/bin/bash
# Round 5, after get-first and the following sender: does a second Range
# stream for the 10 MiB job (a 5 MiB bounded probe + the rest) pay now?
# (r05_split_ab said no, when the PUT trailed the GET by 0.5 ms.)
set -o pipefail
OUT=${OUT:-gpurun_out/r05_get2_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b default_$i &&
  b get2_$i --probe-kb 5120 --http-segments 2 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1)"
done
exit $rc
