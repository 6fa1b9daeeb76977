#!/bin/bash
# Round 5: signed PUT sender, a header send + sendfile per 64 KiB frame
# (default) vs every ready frame in one writev from the file mapping
# (TRITONDL_ZC_WRITE_BATCH=N).  Alternated 300-job runs with the data-plane trace.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_batch_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3 4; do
  b sendfile_$i &&
  TRITONDL_ZC_WRITE_BATCH=16 b batch16_$i &&
  TRITONDL_ZC_WRITE_BATCH=64 b batch64_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1) $(grep -o '"worker_send": [0-9.]*' $f | head -1)"
done
exit $rc
