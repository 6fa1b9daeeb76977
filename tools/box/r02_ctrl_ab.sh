#!/bin/bash
# A/B: previous commit (ab_old/, a copy of the package) vs the request fast path, alternated.
set -o pipefail
OUT=gpurun_out/r02_ctrl_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then B=ab_old/bench.py; else B=bench.py; fi
    timeout -k 10 200 python $B --steps 300 --warmup 10 > $OUT/${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/*.log; do echo "== $f"; grep -o '"value": [0-9.]*' $f | head -1; grep -o '"job_spans_ms_p50[^}]*' $f; done
exit $rc
