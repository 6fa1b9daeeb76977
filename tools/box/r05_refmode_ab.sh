#!/bin/bash
# Round 5: the reference's mode (cleanup off: every job writes a new file, as the
# reference never deletes).  Does mapping the signed PUT's whole file up front
# (TRITONDL_ZC_POPULATE=1) pay there, where the pages are new?  Alternated
# 300-job traced runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_refmode_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode --cleanup off "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b default_$i &&
  TRITONDL_ZC_POPULATE=1 b populate_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1) $(grep -o '"pgfault_per_job": [0-9.]*' $f | head -1)"
done
exit $rc
