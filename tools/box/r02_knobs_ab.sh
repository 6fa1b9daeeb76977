#!/bin/bash
# A/B of data-plane knobs on the 10 MiB headline job (http).
set -o pipefail
OUT=gpurun_out/r02_knobs_ab
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 200 python -u bench.py --steps 300 --warmup 10 --no-gpu-probe "$@"; }
run > $OUT/base.log 2>&1 &&
run --probe-kb 5120 --http-segments 2 > $OUT/probe5m_seg2.log 2>&1 &&
run --probe-kb 3584 --http-segments 3 > $OUT/probe3_5m_seg3.log 2>&1 &&
run --sign-threads 8 > $OUT/sign8.log 2>&1 &&
run --sign-threads 2 > $OUT/sign2.log 2>&1 &&
TRITONDL_TRACE=1 timeout -k 10 300 python -u tools/bench_breakdown.py --reps 60 > $OUT/breakdown.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('value'), d.get('job_spans_ms_p50') or d.get('job'))"; done
exit $rc
