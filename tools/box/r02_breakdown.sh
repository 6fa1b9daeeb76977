#!/bin/bash
# Stage breakdown of the headline job (http and https) with the data-plane trace.
set -o pipefail
OUT=gpurun_out/r02_breakdown
mkdir -p $OUT
export TMPDIR=/tmp
TRITONDL_TRACE=1 timeout -k 10 300 python -u tools/bench_breakdown.py --reps 40 > $OUT/breakdown_http.log 2>&1 &&
TRITONDL_TRACE=1 timeout -k 10 300 python -u tools/bench_breakdown.py --reps 40 --tls > $OUT/breakdown_https.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | tail -2; done
exit $rc
