#!/bin/bash
# Round 5: what bounds the 10 MiB headline job after the fetch ends?  The upload
# trails the download by ~0.8 ms (job spans).  Alternated 300-job runs:
# defaults; unsigned payload (no chunk signing in the worker, no verify in the
# fake); the fake S3 with 8 verifier threads; 8 sign threads in the worker;
# content check off; fakes spread over two CCDs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_bound}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2; do
  b default_$i &&
  b unsigned_$i --payload unsigned &&
  TRITONDL_FAKE_S3_VERIFY_THREADS=8 b verify8_$i &&
  b sign8_$i --sign-threads 8 &&
  b nocheck_$i --no-content-check &&
  b sign2_$i --sign-threads 2 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f | head -1) $(grep -o '"cpu_ms_per_job": {[^}]*}' $f | head -1)"
done
exit $rc
