#!/bin/bash
# Pinned headline: is the upload tail the worker's hashing or the fake S3's
# verification?  Fake S3 verifier threads 4 (default) vs 8, and worker chunk
# hashers 4 (default) vs 6, alternated x2.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_sink_ab}
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in f4s4 f8s4 f8s6 f4s6; do
    f=${v:1:1}; s=${v:3:1}
    TRITONDL_FAKE_S3_VERIFY_THREADS=$f timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --sign-threads $s > $OUT/bench_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/bench_*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_spans_ms_p50[^}]*' $f)"
done
exit $rc
