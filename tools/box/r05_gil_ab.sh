#!/bin/bash
# Round 5: does the GET pump wait on the GIL?  Alternated 300-job runs with the
# data-plane trace: default; a 0.5 ms GIL switch interval (default 5 ms); the
# GET pump launched two loop turns before the streamed upload's first step;
# both.  (Result: get-first 427.7 vs 395.1 jobs/s, now the default; the switch
# interval changed nothing and its knob, TRITONDL_SWITCH_INTERVAL_US, was removed.)
set -o pipefail
OUT=${OUT:-gpurun_out/r05_gil_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b base_$i &&
  TRITONDL_SWITCH_INTERVAL_US=500 b sw500_$i &&
  TRITONDL_GET_FIRST=2 b getfirst_$i &&
  TRITONDL_GET_FIRST=2 TRITONDL_SWITCH_INTERVAL_US=500 b both_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1)"
done
exit $rc
