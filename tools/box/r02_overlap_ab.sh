#!/bin/bash
# Overlapped receive pump (recv and pwrite on two threads) vs sequential
# (TRITONDL_RELAY_OVERLAP=0), headline bench alternated, plus the 1 GiB job.
set -o pipefail
OUT=gpurun_out/r02_overlap_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2 3; do
  for v in seq ovl; do
    if [ $v = seq ]; then export TRITONDL_RELAY_OVERLAP=0; else export TRITONDL_RELAY_OVERLAP=1; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for v in seq ovl; do
  if [ $v = seq ]; then export TRITONDL_RELAY_OVERLAP=0; else export TRITONDL_RELAY_OVERLAP=1; fi
  [ $rc -eq 0 ] && { timeout -k 10 200 python bench.py --steps 20 --warmup 2 --file-mb 1024 > $OUT/${v}_1g.log 2>&1 || rc=$?; }
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_spans_ms_p50[^}]*' $f)"; done
exit $rc
