#!/bin/bash
# Round 5: a single-stream job's fetch runs inline in the downloader's task
# (its pump starts one loop turn after the job's start returns) and the
# worker takes an already-received delivery without racing getter/stopper
# tasks.  Default vs the upload-first order, alternated 300-job traced runs.
# (Result: with the fetch inline the download task runs first either way;
# 406 vs 401 jobs/s, within noise, so the TRITONDL_GET_FIRST knob was removed.)
set -o pipefail
OUT=${OUT:-gpurun_out/r05_inline_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3 4; do
  b default_$i &&
  TRITONDL_GET_FIRST=0 b uploadfirst_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f | head -1)"
done
exit $rc
