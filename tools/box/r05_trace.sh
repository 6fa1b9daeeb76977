#!/bin/bash
# Round 5: data-plane event trace of the headline job (TRITONDL_TRACE=1): when
# the GET pump ends, when the PUT pump has sent its last byte, when S3 answers.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_trace}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2; do
  b default_$i && b unsigned_$i --payload unsigned && b conc2_$i --concurrency 2 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f | head -1)"
done
exit $rc
