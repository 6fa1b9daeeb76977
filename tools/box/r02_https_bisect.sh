#!/bin/bash
# https headline regression hunt: snapshots ab_a (2b55854), ab_b (9220c47), HEAD.
set -o pipefail
OUT=gpurun_out/r02_https_bisect
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in a b head; do
    if [ $v = head ]; then B=bench.py; else B=ab_$v/bench.py; fi
    timeout -k 10 200 python $B --steps 300 --warmup 10 --tls --no-gpu-probe > $OUT/${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_spans_ms_p50[^}]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f)"; done
exit $rc
