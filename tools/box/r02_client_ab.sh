#!/bin/bash
# AMQP client callback reads: ab_old (task-based reader) vs current, headline alternated.
set -o pipefail
OUT=gpurun_out/r02_client_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then B=ab_old/bench.py; else B=bench.py; fi
    timeout -k 10 200 python $B --steps 300 --warmup 10 --no-gpu-probe > $OUT/${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"publish": [0-9.]*, "ack": [0-9.]*' $f)"; done
exit $rc
