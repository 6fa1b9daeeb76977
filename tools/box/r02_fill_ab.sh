#!/bin/bash
# 256 KiB flow granularity in the receive pump; sign threads 4 vs 8; http + https.
set -o pipefail
OUT=gpurun_out/r02_fill_ab
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u bench.py --steps 300 --warmup 10 --no-gpu-probe "$@"; }
run > $OUT/fill256_sign4.log 2>&1 &&
run --sign-threads 8 > $OUT/fill256_sign8.log 2>&1 &&
run --sign-threads 6 > $OUT/fill256_sign6.log 2>&1 &&
run --tls > $OUT/fill256_https.log 2>&1 &&
TRITONDL_TRACE=1 timeout -k 10 300 python -u tools/bench_breakdown.py --reps 60 > $OUT/breakdown.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('value'), d.get('job_spans_ms_p50') or d.get('job'))"; done
exit $rc
