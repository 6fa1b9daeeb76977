#!/bin/bash
# Headline after the fast HMAC chain (sign threads default = half the CPUs).
set -o pipefail
OUT=gpurun_out/r02_hmac
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u bench.py --steps 300 --warmup 10 --no-gpu-probe "$@"; }
run > $OUT/http_a.log 2>&1 && run > $OUT/http_b.log 2>&1 && run --tls > $OUT/https.log 2>&1 &&
run --tls --payload streaming > $OUT/https_chunked.log 2>&1 &&
TRITONDL_TRACE=1 timeout -k 10 300 python -u tools/bench_breakdown.py --reps 60 > $OUT/breakdown.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('value'), d.get('config',{}).get('s3_sign_threads'), d.get('job_spans_ms_p50') or d.get('job'))"; done
exit $rc
