#!/bin/bash
# https headline: parallel TLS range streams (decrypt on several cores) A/B.
set -o pipefail
OUT=gpurun_out/r02_tls_ab
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u bench.py --steps 300 --warmup 10 --no-gpu-probe --tls "$@"; }
run > $OUT/base.log 2>&1 &&
run --probe-kb 5120 --http-segments 2 > $OUT/p5m_s2.log 2>&1 &&
run --probe-kb 3584 --http-segments 3 > $OUT/p3_5m_s3.log 2>&1 &&
run --probe-kb 2560 --http-segments 4 > $OUT/p2_5m_s4.log 2>&1 &&
run > $OUT/base2.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('value'), d.get('cpu_ms_per_job'), d.get('job_spans_ms_p50'))"; done
exit $rc
