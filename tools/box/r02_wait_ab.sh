#!/bin/bash
# Headline A/B: harness waits via futures (HEAD) vs 1 ms polling (ab_old = HEAD~1), alternated.
set -o pipefail
OUT=gpurun_out/r02_wait_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2 3; do
  for v in old head; do
    if [ $v = head ]; then B=bench.py; else B=ab_old/bench.py; fi
    timeout -k 10 200 python $B --steps 300 --warmup 10 --no-gpu-probe > $OUT/${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f)"; done
exit $rc
