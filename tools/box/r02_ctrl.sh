#!/bin/bash
# Headline after the request fast path: 3 x bench (300 steps) + traced breakdown.
set -o pipefail
OUT=gpurun_out/r02_ctrl
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/bench_a.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/bench_b.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/bench_c.log 2>&1 &&
TRITONDL_TRACE=1 timeout -k 10 200 python tools/bench_breakdown.py --reps 100 > $OUT/breakdown.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --tls --no-gpu-probe > $OUT/bench_https.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | tail -1 | cut -c1-300; grep -o '"job_spans_ms_p50.*' $f | cut -c1-200; done
grep -o '"trace_ms_p50.*' $OUT/breakdown.log
exit $rc
