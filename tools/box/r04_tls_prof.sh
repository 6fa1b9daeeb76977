#!/bin/bash
# https headline: where the worker's CPU goes (sampled profile) and the stage spans.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_tls_prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --tls --cpuprofile $OUT/tls.prof > $OUT/bench_tls.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_http.log 2>&1
python tools/bench_summary.py $OUT/bench_tls.log $OUT/bench_http.log
grep -o '"job_spans_ms_p50": {[^}]*}' $OUT/bench_tls.log $OUT/bench_http.log
head -40 $OUT/tls.prof.txt
